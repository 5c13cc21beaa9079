"""ctypes binding of the batched ROS1 wire adapters (include/wbc_ros.h, libwbc_ros.so).

Host-only (the library has no HIP dependency).  Decoders take a list of B serialized messages
(bytes) and return the engine's input arrays; encoders take the engine's output arrays and return
B serialized messages.  Errors raise WbcError with the library's message (robot index + field).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._capi import NU_LEN, NUM_JOINTS, POSE_LEN, REF_LEN, WbcError

HERE = os.path.dirname(os.path.abspath(__file__))
ROS_LIB_PATH = os.path.join(HERE, "libwbc_ros.so")

# every entry point declared in include/wbc_ros.h
ROS_API_SYMBOLS = ["wbc_ros_md5sum", "wbc_ros_last_error", "wbc_ros_decode_reference", "wbc_ros_decode_model_states",
                   "wbc_ros_decode_joint_state", "wbc_ros_decode_twist", "wbc_ros_encode_float64_array",
                   "wbc_ros_encode_reference"]

REFERENCE_MSG_LEN = 508  # 6 Float64MultiArray (12-byte header each) + 54 doubles + bool[4]

_lib = None


def load_ros_library(path: str = ROS_LIB_PATH):
    global _lib
    if _lib is None:
        lib = C.CDLL(path)
        P, I32, U64 = C.c_void_p, C.c_int32, C.c_uint64
        sigs = {
            "wbc_ros_md5sum": ([C.c_char_p], C.c_char_p),
            "wbc_ros_last_error": ([], C.c_char_p),
            "wbc_ros_decode_reference": ([P, P, I32, P, P], I32),
            "wbc_ros_decode_model_states": ([P, P, I32, C.c_char_p, P, P], I32),
            "wbc_ros_decode_joint_state": ([P, P, I32, P, P, P], I32),
            "wbc_ros_decode_twist": ([P, P, I32, P], I32),
            "wbc_ros_encode_float64_array": ([P, I32, I32, P, U64, C.POINTER(U64)], I32),
            "wbc_ros_encode_reference": ([P, P, I32, P, U64, C.POINTER(U64)], I32),
        }
        for name, (args, res) in sigs.items():
            f = getattr(lib, name)
            f.argtypes, f.restype = args, res
        _lib = lib
    return _lib


def md5sum(datatype: str) -> str | None:
    r = load_ros_library().wbc_ros_md5sum(datatype.encode())
    return None if r is None else r.decode()


def _check(rc, what):
    if rc != 0:
        raise WbcError(f"{what} failed ({rc}): {load_ros_library().wbc_ros_last_error().decode()}")


def _msg_arrays(msgs):
    """Keep the buffers alive for the call: (pointer array, length array, owners)."""
    bufs = [C.create_string_buffer(bytes(m), max(len(m), 1)) for m in msgs]
    ptrs = (C.c_void_p * max(len(bufs), 1))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_uint64 * max(len(bufs), 1))(*[len(m) for m in msgs])
    return ptrs, lens, bufs


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def decode_reference(msgs):
    """B WbcReferenceMsg -> (ref [B, 54], contacts [B] uint8 bitmask) (referenceCallback, cpp:150-185)."""
    B = len(msgs)
    ref, con = np.zeros((B, REF_LEN)), np.zeros(B, np.uint8)
    ptrs, lens, _keep = _msg_arrays(msgs)
    _check(load_ros_library().wbc_ros_decode_reference(ptrs, lens, B, _p(ref), _p(con)), "wbc_ros_decode_reference")
    return ref, con


def decode_model_states(msgs, model_name: str | None = None, nu=None):
    """B ModelStates -> (base_pose [B, 7], nu [B, 18] with entries 0..5 filled)."""
    B = len(msgs)
    pose = np.zeros((B, POSE_LEN))
    nu = np.zeros((B, NU_LEN)) if nu is None else nu
    ptrs, lens, _keep = _msg_arrays(msgs)
    _check(load_ros_library().wbc_ros_decode_model_states(ptrs, lens, B, model_name.encode() if model_name else None,
                                                          _p(pose), _p(nu)), "wbc_ros_decode_model_states")
    return pose, nu


def decode_joint_state(msgs, joint_names=None, nu=None):
    """B JointState -> (qj [B, 12], nu [B, 18] with entries 6..17 filled), model joint order."""
    B = len(msgs)
    qj = np.zeros((B, NUM_JOINTS))
    nu = np.zeros((B, NU_LEN)) if nu is None else nu
    names = None
    if joint_names is not None:
        enc = [n.encode() for n in joint_names]
        names = (C.c_char_p * NUM_JOINTS)(*enc)
    ptrs, lens, _keep = _msg_arrays(msgs)
    _check(load_ros_library().wbc_ros_decode_joint_state(ptrs, lens, B, C.cast(names, C.c_void_p) if names else None,
                                                         _p(qj), _p(nu)), "wbc_ros_decode_joint_state")
    return qj, nu


def decode_twist(msgs):
    """B Twist -> cmd [B, 3] = (linear.x, linear.y, angular.z) (MotionPlanner::input_callback)."""
    B = len(msgs)
    cmd = np.zeros((B, 3))
    ptrs, lens, _keep = _msg_arrays(msgs)
    _check(load_ros_library().wbc_ros_decode_twist(ptrs, lens, B, _p(cmd)), "wbc_ros_decode_twist")
    return cmd


def encode_float64_array(rows):
    """[B, n] -> B Float64MultiArray messages (the torque / GRF publishers, cpp:558-576)."""
    rows = np.ascontiguousarray(rows, np.float64)
    B, n = rows.shape
    L = 12 + 8 * n
    out = np.zeros(max(B, 1) * L, np.uint8)
    ml = C.c_uint64()
    _check(load_ros_library().wbc_ros_encode_float64_array(_p(rows), B, n, _p(out), L, C.byref(ml)),
           "wbc_ros_encode_float64_array")
    assert ml.value == L
    return [out[b * L:(b + 1) * L].tobytes() for b in range(B)]


def encode_reference(ref, contacts):
    """ref [B, 54] + contacts [B] -> B WbcReferenceMsg messages (the planner's publisher)."""
    ref = np.ascontiguousarray(ref, np.float64)
    con = np.ascontiguousarray(contacts, np.uint8)
    B = ref.shape[0]
    L = REFERENCE_MSG_LEN
    out = np.zeros(max(B, 1) * L, np.uint8)
    ml = C.c_uint64()
    _check(load_ros_library().wbc_ros_encode_reference(_p(ref), _p(con), B, _p(out), L, C.byref(ml)),
           "wbc_ros_encode_reference")
    assert ml.value == L
    return [out[b * L:(b + 1) * L].tobytes() for b in range(B)]
