"""ctypes binding of the C-ABI in include/wbc.h (libwbc_hip.so, built in-tree).

There is no CPU fallback: if the HIP library is missing or no GPU is present, loading or
creating an engine raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WBC_LIB", os.path.join(HERE, "libwbc_hip.so"))

NUM_JOINTS, NV, NC = 12, 42, 70
POSE_LEN, NU_LEN, REF_LEN = 7, 18, 54
STATELESS, DEBUG, NO_X, SPLIT, TIMED, COLD, FUSED, GROUP, RESIDENT = 1, 2, 4, 8, 16, 32, 64, 128, 256
QP_OK, QP_MAX_ITER, QP_INFEASIBLE, QP_NUMERIC = 0, 1, 2, 3

# WBC_DBG_* offsets (include/wbc.h)
DBG = dict(COM=0, COMVEL=3, POSE=6, VC=12, M=18, CNU=342, JFEET=360, PFEET=576, VFEET=588, MBARB=600, MBARJ=636,
           JBAR=780, BBAR=996, WRENCH=1014, R1=1020, RSW=1032, STAMPS=1044, LEN=1052)

# every entry point declared in include/wbc.h
C_API_SYMBOLS = [
    "wbc_default_params", "wbc_anymal_model", "wbc_create", "wbc_destroy", "wbc_batch", "wbc_set_stream",
    "wbc_set_state", "wbc_set_reference", "wbc_bind_device_inputs", "wbc_bind_device_outputs", "wbc_reset", "wbc_update", "wbc_solve",
    "wbc_step", "wbc_set_modes", "wbc_step_modes", "wbc_modes_per_wave", "wbc_cycle", "wbc_synchronize", "wbc_get_output", "wbc_device_outputs", "wbc_get_debug", "wbc_last_kernel_ms",
    "wbc_last_error", "wbc_model_from_urdf",
]


class WbcLink(C.Structure):
    _fields_ = [("R", C.c_double * 9), ("p", C.c_double * 3), ("axis", C.c_double * 3), ("mass", C.c_double),
                ("com", C.c_double * 3), ("inertia", C.c_double * 9)]


class WbcModel(C.Structure):
    _fields_ = [("base_mass", C.c_double), ("base_com", C.c_double * 3), ("base_inertia", C.c_double * 9),
                ("link", (WbcLink * 3) * 4), ("foot", (C.c_double * 3) * 4), ("total_mass", C.c_double)]


class WbcParams(C.Structure):
    _fields_ = [("friction", C.c_double), ("loop_rate", C.c_double), ("max_torque", C.c_double),
                ("kp", C.c_double), ("kp_z", C.c_double), ("kd", C.c_double), ("ki", C.c_double),
                ("kp_swing", C.c_double), ("kd_swing", C.c_double), ("slack_weight", C.c_double),
                ("initial_reference_pose", C.c_double * 6), ("gravity", C.c_double), ("max_wsr", C.c_int32),
                ("reserved", C.c_int32)]


_lib = None


def load_library(path: str = LIB_PATH):
    """Load libwbc_hip.so (raises OSError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"HIP engine library not built: {path} (run __graft_entry__.build())")
    # One HIP runtime per process: torch bundles its own libamdhip64 (soname libamdhip64.so.7,
    # requested as "libamdhip64.so").  Loaded first, it satisfies our DT_NEEDED
    # libamdhip64.so.7 and both share it; loaded after us, it would be mapped a second time and
    # torch's device init fails ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    P, I32, U32 = C.c_void_p, C.c_int32, C.c_uint32
    dp = C.POINTER(C.c_double)
    sig = {
        "wbc_default_params": ([C.POINTER(WbcParams)], I32),
        "wbc_anymal_model": ([C.POINTER(WbcModel)], I32),
        "wbc_create": ([C.POINTER(WbcModel), C.POINTER(WbcParams), I32, I32, C.POINTER(P)], I32),
        "wbc_destroy": ([P], I32),
        "wbc_batch": ([P], I32),
        "wbc_set_stream": ([P, P], I32),
        "wbc_set_state": ([P, P, P, P], I32),
        "wbc_set_reference": ([P, P, P, P], I32),
        "wbc_bind_device_inputs": ([P, P, P, P, P, P, P], I32),
        "wbc_bind_device_outputs": ([P, P, P, P, P, P], I32),
        "wbc_reset": ([P, P], I32),
        "wbc_update": ([P, U32], I32),
        "wbc_solve": ([P, U32], I32),
        "wbc_step": ([P, U32], I32),
        "wbc_set_modes": ([P, I32, P], I32),
        "wbc_cycle": ([P, P, P, P, P, P, P, U32, P, P, P, P, P], I32),
        "wbc_step_modes": ([P, U32], I32),
        "wbc_modes_per_wave": ([P, C.POINTER(C.c_int32)], I32),
        "wbc_synchronize": ([P], I32),
        "wbc_get_output": ([P, P, P, P, P, P], I32),
        "wbc_device_outputs": ([P, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P)], I32),
        "wbc_get_debug": ([P, P], I32),
        "wbc_last_kernel_ms": ([P, dp], I32),
        "wbc_last_error": ([], C.c_char_p),
        "wbc_model_from_urdf": ([C.c_char_p, P, P, C.c_char_p, C.POINTER(WbcModel)], I32),
    }
    for name, (argt, rest) in sig.items():
        if name == "wbc_modes_per_wave" and not hasattr(lib, name):
            continue  # a diagnostic entry point: earlier builds (A/B variants, tools/build_rev.sh) lack it
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = rest
    _lib = lib
    return lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def default_params() -> WbcParams:
    p = WbcParams()
    load_library().wbc_default_params(C.byref(p))
    return p


def model_from_urdf(path: str, legs=None, joints=None, foot_suffix=None) -> WbcModel:
    """wbc_model_from_urdf: lumped 12-DoF quadruped model from a URDF file (raises WbcError)."""
    lib = load_library()

    def names(v):
        if v is None:
            return None
        arr = (C.c_char_p * len(v))(*[x.encode() for x in v])
        return C.cast(arr, C.c_void_p), arr

    m = WbcModel()
    lg, jn = names(legs), names(joints)
    rc = lib.wbc_model_from_urdf(path.encode(), lg[0] if lg else None, jn[0] if jn else None,
                                 foot_suffix.encode() if foot_suffix else None, C.byref(m))
    if rc != 0:
        raise WbcError(f"wbc_model_from_urdf failed ({rc}): {lib.wbc_last_error().decode()}")
    return m


def anymal_model() -> WbcModel:
    m = WbcModel()
    load_library().wbc_anymal_model(C.byref(m))
    return m


class WbcError(RuntimeError):
    pass


class Engine:
    """A batch of B robots on one GPU (wraps wbc_engine*)."""

    def __init__(self, batch: int, device: int = 0, params: WbcParams | None = None, model: WbcModel | None = None):
        self.lib = load_library()
        self.batch = int(batch)
        self.n_modes = 0
        self._stream = None  # the bound caller stream object (kept alive while bound)
        self.h = C.c_void_p()
        rc = self.lib.wbc_create(C.byref(model) if model else None, C.byref(params) if params else None,
                                 self.batch, int(device), C.byref(self.h))
        self._check(rc, "wbc_create")

    def _check(self, rc, what):
        if rc != 0:
            raise WbcError(f"{what} failed ({rc}): {self.lib.wbc_last_error().decode()}")

    def close(self):
        if self.h:
            self.lib.wbc_destroy(self.h)  # synchronizes the bound stream, which is still alive here
            self.h = C.c_void_p()
        self._stream = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- inputs -------------------------------------------------------------------------
    @property
    def input_rows(self) -> int:
        """Rows of the input arrays: B robots, or B / K states under K mode hypotheses."""
        return self.batch // self.n_modes if self.n_modes else self.batch

    def set_state(self, base_pose=None, nu=None, qj=None):
        B = self.input_rows
        arrs = [None if v is None else np.ascontiguousarray(v, np.float64).reshape(B, n)
                for v, n in ((base_pose, POSE_LEN), (nu, NU_LEN), (qj, NUM_JOINTS))]
        self._check(self.lib.wbc_set_state(self.h, *[_ptr(a) for a in arrs]), "wbc_set_state")

    def set_reference(self, ref=None, contacts=None, switching=None):
        B = self.input_rows
        r = None if ref is None else np.ascontiguousarray(ref, np.float64).reshape(B, REF_LEN)
        c = None if contacts is None else np.ascontiguousarray(contacts, np.uint8).reshape(B)
        s = None if switching is None else np.ascontiguousarray(switching, np.uint8).reshape(B)
        self._check(self.lib.wbc_set_reference(self.h, _ptr(r), _ptr(c), _ptr(s)), "wbc_set_reference")

    def bind_device_inputs(self, base_pose=0, nu=0, qj=0, ref=0, contacts=0, switching=0):
        """Integer device pointers (e.g. torch tensor .data_ptr()); 0 = engine-owned buffer."""
        v = [C.c_void_p(int(x)) if x else None for x in (base_pose, nu, qj, ref, contacts, switching)]
        self._check(self.lib.wbc_bind_device_inputs(self.h, *v), "wbc_bind_device_inputs")

    def bind_device_outputs(self, tau=0, grf=0, x=0, status=0, iters=0):
        """Integer device pointers of caller-owned output buffers; 0 = engine-owned buffer."""
        v = [C.c_void_p(int(p)) if p else None for p in (tau, grf, x, status, iters)]
        self._check(self.lib.wbc_bind_device_outputs(self.h, *v), "wbc_bind_device_outputs")

    def set_stream(self, stream):
        """Bind a caller stream: a torch.cuda.Stream (or any object with `cuda_stream`), which the engine
        keeps referenced until it is unbound (set_stream(0 / None)) or closed, so the stream outlives
        its binding (include/wbc.h wbc_set_stream); or a raw hipStream_t as an int, which the caller
        must keep alive that long.  0 / None: the engine's own stream."""
        ptr = int(getattr(stream, "cuda_stream", stream) or 0)
        self._check(self.lib.wbc_set_stream(self.h, C.c_void_p(ptr) if ptr else None), "wbc_set_stream")
        self._stream = stream if ptr else None

    # --- execution ----------------------------------------------------------------------
    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8).reshape(self.batch)
        self._check(self.lib.wbc_reset(self.h, _ptr(m)), "wbc_reset")

    def update(self, flags: int = 0):
        self._check(self.lib.wbc_update(self.h, flags), "wbc_update")

    def solve(self, flags: int = 0):
        self._check(self.lib.wbc_solve(self.h, flags), "wbc_solve")

    def step(self, flags: int = 0):
        self._check(self.lib.wbc_step(self.h, flags), "wbc_step")

    def cycle(self, base_pose, nu, qj, ref, contacts, switching, flags: int = 0, want_x: bool = True):
        """wbc_cycle: one synchronous host-to-host control cycle (one H2D copy, the step, one D2H copy)."""
        B = self.batch
        f = lambda v, n: np.ascontiguousarray(v, np.float64).reshape(B, n)
        ins = [f(base_pose, POSE_LEN), f(nu, NU_LEN), f(qj, NUM_JOINTS), f(ref, REF_LEN),
               np.ascontiguousarray(contacts, np.uint8).reshape(B), np.ascontiguousarray(switching, np.uint8).reshape(B)]
        tau = np.zeros((B, NUM_JOINTS)); grf = np.zeros((B, NUM_JOINTS)); x = np.zeros((B, NV)) if want_x else None
        st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
        self._check(self.lib.wbc_cycle(self.h, *[_ptr(a) for a in ins], flags, _ptr(tau), _ptr(grf), _ptr(x), _ptr(st),
                                       _ptr(it)), "wbc_cycle")
        return dict(tau=tau, grf=grf, x=x, status=st, iters=it)

    def set_modes(self, modes=None):
        """wbc_set_modes: solve every state under each contact mask in `modes` (None / [] clears)."""
        m = None if modes is None or len(modes) == 0 else np.ascontiguousarray(modes, np.uint8).ravel()
        n = 0 if m is None else m.size
        self._check(self.lib.wbc_set_modes(self.h, n, _ptr(m)), "wbc_set_modes")
        self.n_modes = n

    def step_modes(self, flags: int = 1):
        """wbc_step_modes: one cold step of every (state, mode) hypothesis (flags need STATELESS)."""
        self._check(self.lib.wbc_step_modes(self.h, flags), "wbc_step_modes")

    def modes_per_wave(self) -> int:
        """wbc_modes_per_wave: hypotheses per wave of wbc_step_modes (1: one per segment; M > 1: the
        mode loop, wbc_modes_kernel); 0 without modes."""
        m = C.c_int32(0)
        self._check(self.lib.wbc_modes_per_wave(self.h, C.byref(m)), "wbc_modes_per_wave")
        return int(m.value)

    def synchronize(self):
        self._check(self.lib.wbc_synchronize(self.h), "wbc_synchronize")

    def last_kernel_ms(self) -> float:
        ms = C.c_double()
        self._check(self.lib.wbc_last_kernel_ms(self.h, C.byref(ms)), "wbc_last_kernel_ms")
        return ms.value

    # --- outputs ------------------------------------------------------------------------
    def outputs(self):
        B = self.batch
        tau = np.zeros((B, NUM_JOINTS)); grf = np.zeros((B, NUM_JOINTS)); x = np.zeros((B, NV))
        st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
        self._check(self.lib.wbc_get_output(self.h, _ptr(tau), _ptr(grf), _ptr(x), _ptr(st), _ptr(it)),
                    "wbc_get_output")
        return dict(tau=tau, grf=grf, x=x, status=st, iters=it)

    def device_outputs(self):
        ptrs = [C.c_void_p() for _ in range(5)]
        self._check(self.lib.wbc_device_outputs(self.h, *[C.byref(p) for p in ptrs]), "wbc_device_outputs")
        return dict(zip(("tau", "grf", "x", "status", "iters"), (p.value for p in ptrs)))

    def debug(self):
        out = np.zeros((self.batch, DBG["LEN"]))
        self._check(self.lib.wbc_get_debug(self.h, _ptr(out)), "wbc_get_debug")
        return out


def split_debug(rec):
    """Debug record (WBC_DBG_LEN,) -> dict of named arrays (same keys as oracle debug_record)."""
    D = DBG
    return dict(com=rec[D["COM"]:D["COM"] + 3], comvel=rec[D["COMVEL"]:D["COMVEL"] + 3],
                pose=rec[D["POSE"]:D["POSE"] + 6], vc=rec[D["VC"]:D["VC"] + 6],
                M=rec[D["M"]:D["M"] + 324].reshape(18, 18), Cnu=rec[D["CNU"]:D["CNU"] + 18],
                Jfeet=rec[D["JFEET"]:D["JFEET"] + 216].reshape(12, 18), pfeet=rec[D["PFEET"]:D["PFEET"] + 12],
                vfeet=rec[D["VFEET"]:D["VFEET"] + 12], Mbar_b=rec[D["MBARB"]:D["MBARB"] + 36].reshape(6, 6),
                Mbar_j=rec[D["MBARJ"]:D["MBARJ"] + 144].reshape(12, 12),
                Jbar=rec[D["JBAR"]:D["JBAR"] + 216].reshape(12, 18), bbar=rec[D["BBAR"]:D["BBAR"] + 18],
                W=rec[D["WRENCH"]:D["WRENCH"] + 6], r1=rec[D["R1"]:D["R1"] + 12], rsw=rec[D["RSW"]:D["RSW"] + 12])


# --- batched motion planner (include/wbc_planner.h) -----------------------------------------------
class WbcPlannerParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("step_length", "height_control_point", "x_offset", "y_offset",
                                          "step_duration", "body_height", "body_initial_velocity",
                                          "body_final_velocity", "dt")]


PLANNER_API_SYMBOLS = ["wbc_planner_default_params", "wbc_planner_create", "wbc_planner_destroy",
                       "wbc_planner_set_stream", "wbc_planner_set_command", "wbc_planner_reset", "wbc_planner_tick",
                       "wbc_planner_device_outputs", "wbc_planner_get_output"]


def _planner_lib():
    lib = load_library()
    if not getattr(lib, "_planner_sigs", False):
        P, I32 = C.c_void_p, C.c_int32
        PP = C.POINTER(P)
        sig = {
            "wbc_planner_default_params": ([C.POINTER(WbcPlannerParams)], I32),
            "wbc_planner_create": ([C.POINTER(WbcPlannerParams), I32, I32, C.POINTER(P)], I32),
            "wbc_planner_destroy": ([P], I32),
            "wbc_planner_set_stream": ([P, P], I32),
            "wbc_planner_set_command": ([P, P], I32),
            "wbc_planner_reset": ([P, P], I32),
            "wbc_planner_tick": ([P], I32),
            "wbc_planner_device_outputs": ([P, PP, PP, PP, PP], I32),
            "wbc_planner_get_output": ([P, P, P, P, P], I32),
        }
        for name, (argt, rest) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = argt
            fn.restype = rest
        lib._planner_sigs = True
    return lib


class Planner:
    """B motion planners on one GPU (wraps wbc_planner*): one tick = one plannerLoop rate.sleep()."""

    def __init__(self, batch: int, device: int = 0, params: WbcPlannerParams | None = None):
        self.lib = _planner_lib()
        self.batch = int(batch)
        self.h = C.c_void_p()
        rc = self.lib.wbc_planner_create(C.byref(params) if params else None, self.batch, int(device), C.byref(self.h))
        self._check(rc, "wbc_planner_create")

    def _check(self, rc, what):
        if rc != 0:
            raise WbcError(f"{what} failed ({rc}): {self.lib.wbc_last_error().decode()}")

    def close(self):
        if self.h:
            self.lib.wbc_planner_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr: int):
        self._check(self.lib.wbc_planner_set_stream(self.h, C.c_void_p(int(stream_ptr)) if stream_ptr else None),
                    "wbc_planner_set_stream")

    def set_command(self, cmd):
        c = np.ascontiguousarray(cmd, np.float64).reshape(self.batch, 3)
        self._check(self.lib.wbc_planner_set_command(self.h, _ptr(c)), "wbc_planner_set_command")

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8).reshape(self.batch)
        self._check(self.lib.wbc_planner_reset(self.h, _ptr(m)), "wbc_planner_reset")

    def tick(self):
        self._check(self.lib.wbc_planner_tick(self.h), "wbc_planner_tick")

    def device_outputs(self):
        p = [C.c_void_p() for _ in range(4)]
        self._check(self.lib.wbc_planner_device_outputs(self.h, *[C.byref(x) for x in p]), "wbc_planner_device_outputs")
        return dict(zip(("ref", "contacts", "switching", "published"), (x.value for x in p)))

    def outputs(self):
        B = self.batch
        ref = np.zeros((B, REF_LEN))
        con, sw, pub = (np.zeros(B, np.uint8) for _ in range(3))
        self._check(self.lib.wbc_planner_get_output(self.h, _ptr(ref), _ptr(con), _ptr(sw), _ptr(pub)),
                    "wbc_planner_get_output")
        return dict(ref=ref, contacts=con, switching=sw, published=pub)
