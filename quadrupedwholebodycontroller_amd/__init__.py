"""quadrupedwholebodycontroller_amd — MI355X-native batched whole-body-control QP engine.

The hot path of the reference's `WholeBodyController` (updateState -> solveQP ->
computeJointTorques, src/whole_body_controller.cpp:650-652) as hand-written HIP for gfx950,
behind the C-ABI in include/wbc.h.  This package is the Python view of that C-ABI:

  Engine          batched handle (wbc_create ... wbc_get_output), see _capi.py
  Planner         batched motion planner (WbcReferenceMsg producer), see _capi.py
  workloads       synthetic inputs of the BASELINE.json configurations
  sharding        robot shards and the per-step all-gather of the multi-GPU path
  ros_wire        ROS1 wire-byte adapters (libwbc_ros.so)

The WholeBodyController-shaped single-robot shim is C++ (include/wbc_controller.hpp,
libwbc_controller.so), as the reference's class is.

The product path has no CPU fallback: without libwbc_hip.so or a GPU it raises.
"""
from ._capi import (COLD, DEBUG, FUSED, GROUP, NO_X, RESIDENT, SPLIT, STATELESS, TIMED, QP_INFEASIBLE, QP_MAX_ITER, QP_NUMERIC, QP_OK, Engine, WbcError,  # noqa: F401
                    WbcModel, WbcParams, anymal_model, default_params, load_library, model_from_urdf, split_debug, Planner,
                    WbcPlannerParams)

__all__ = ["Engine", "Planner", "WbcPlannerParams", "model_from_urdf", "WbcError", "WbcModel", "WbcParams", "anymal_model", "default_params", "load_library",
           "split_debug", "STATELESS", "DEBUG", "NO_X", "SPLIT", "TIMED", "COLD", "FUSED", "GROUP", "RESIDENT", "QP_OK", "QP_MAX_ITER", "QP_INFEASIBLE", "QP_NUMERIC"]
