"""ctypes binding of libfqlpop.so (the C ABI in include/fqlpop.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (``make -C
flow-q-learning_amd/csrc``) and loaded from this directory.  There is no
fallback: if the library is missing or fails to load, every entry point raises.
``torch`` is imported first when available so that the process has ONE HIP
runtime (torch's bundled libamdhip64.so.7 and ROCm's share the soname).
"""
from __future__ import annotations

import ctypes
import os

try:  # share torch's HIP runtime if torch is around (it usually is)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is in the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfqlpop.so")

INFO_STRIDE = 16
TRAIN_INFO_KEYS = (
    "critic/critic_loss", "critic/q_mean", "critic/q_max", "critic/q_min",
    "actor/actor_loss", "actor/bc_flow_loss", "actor/distill_loss",
    "actor/q_loss", "actor/q", "actor/mse",
    "grad/max", "grad/min", "grad/norm",
)
VAL_INFO_KEYS = TRAIN_INFO_KEYS[:10]
STATE_PARAMS, STATE_ADAM_M, STATE_ADAM_V = 0, 1, 2


class FqlpopError(RuntimeError):
    pass


class Config(ctypes.Structure):
    """Mirror of ``fqlpop_config`` (include/fqlpop.h)."""
    _fields_ = [
        ("obs_dim", ctypes.c_int), ("action_dim", ctypes.c_int),
        ("hidden_dim", ctypes.c_int), ("num_hidden", ctypes.c_int),
        ("batch_size", ctypes.c_int), ("num_qs", ctypes.c_int),
        ("layer_norm", ctypes.c_int), ("actor_layer_norm", ctypes.c_int),
        ("flow_steps", ctypes.c_int), ("q_agg_min", ctypes.c_int),
        ("normalize_q_loss", ctypes.c_int),
        ("discount", ctypes.c_float), ("tau", ctypes.c_float), ("lr", ctypes.c_float),
        ("use_graph", ctypes.c_int),
    ]


class EnvModelConfig(ctypes.Structure):
    """Mirror of ``fqlpop_envmodel_config`` (include/fqlpop.h)."""
    _fields_ = [
        ("obs_dim", ctypes.c_int), ("action_dim", ctypes.c_int),
        ("sp_num_hidden", ctypes.c_int), ("sp_hidden", ctypes.c_int * 7),
        ("tp_num_hidden", ctypes.c_int), ("tp_hidden", ctypes.c_int * 7),
    ]


class EmTrainConfig(ctypes.Structure):
    """Mirror of ``fqlpop_emtrain_config`` (include/fqlpop.h)."""
    _fields_ = [
        ("kind", ctypes.c_int), ("obs_dim", ctypes.c_int), ("action_dim", ctypes.c_int),
        ("num_hidden", ctypes.c_int), ("hidden_dims", ctypes.c_int * 8),
        ("batch_size", ctypes.c_int), ("steps", ctypes.c_int),
        ("init_lr", ctypes.c_float), ("termination_weight", ctypes.c_float),
        ("true_termination_weight", ctypes.c_float), ("focal_alpha", ctypes.c_float),
        ("focal_gamma", ctypes.c_float), ("dropout_rate", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("tp_num_hidden", ctypes.c_int), ("tp_hidden_dims", ctypes.c_int * 8),
        ("sequence_length", ctypes.c_int), ("episode_length", ctypes.c_int),
    ]


EM_STATE_PREDICTOR, EM_TERMINATION, EM_MULTISTEP = 0, 1, 2
EM_LOG_STRIDE = 8
_P = ctypes.c_void_p
_F = ctypes.POINTER(ctypes.c_float)
_U8 = ctypes.POINTER(ctypes.c_uint8)
_SIGS = {
    "fqlpop_last_error": (ctypes.c_char_p, []),
    "fqlpop_set_engine_option": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "fqlpop_get_engine_option": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "fqlpop_reset_engine_options": (ctypes.c_int, []),
    "fqlpop_diagnostic_build": (ctypes.c_int, []),
    "fqlpop_step_streams": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "fqlpop_split_plan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_int)]),
    "fqlpop_probe_coverage": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                             ctypes.POINTER(ctypes.c_int64)]),
    "fqlpop_create": (ctypes.c_int, [ctypes.POINTER(Config), ctypes.c_int, _F,
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.c_int,
                                     ctypes.POINTER(_P)]),
    "fqlpop_destroy": (ctypes.c_int, [_P]),
    "fqlpop_set_dataset": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, _P,
                                          ctypes.c_int64, ctypes.c_int]),
    "fqlpop_set_active": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint8)]),
    "fqlpop_step": (ctypes.c_int, [_P, ctypes.c_int]),
    "fqlpop_step_injected": (ctypes.c_int, [_P, _F, _F]),
    "fqlpop_total_loss": (ctypes.c_int, [_P, _F, _F]),
    "fqlpop_read_info": (ctypes.c_int, [_P, ctypes.c_int, _F]),
    "fqlpop_sample_actions": (ctypes.c_int, [_P, ctypes.c_int, _F, ctypes.c_int64, _F,
                                             ctypes.c_uint64, _F]),
    "fqlpop_state_size": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "fqlpop_get_state": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _F, ctypes.c_int64]),
    "fqlpop_set_state": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _F, ctypes.c_int64]),
    "fqlpop_get_count": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]),
    "fqlpop_set_count": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int32]),
    "fqlpop_set_member": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_float, ctypes.c_uint64,
                                         ctypes.c_int]),
    "fqlpop_num_leaves": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int)]),
    "fqlpop_leaf_info": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int64)]),
    "fqlpop_sync": (ctypes.c_int, [_P]),
    "fqlpop_debug_fail_split": (ctypes.c_int, [_P]),
    "fqlpop_time_dominant_kernel": (ctypes.c_int, [_P, ctypes.c_int,
                                                   ctypes.POINTER(ctypes.c_double),
                                                   ctypes.POINTER(ctypes.c_double)]),
    "fqlpop_flops_per_member_step": (ctypes.c_double, [ctypes.POINTER(Config)]),
    "fqlpop_set_probe": (ctypes.c_int, [_P, ctypes.c_int]),
    "fqlpop_dominant_kernel_info": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int,
                                                   ctypes.POINTER(ctypes.c_double),
                                                   ctypes.POINTER(ctypes.c_double)]),
    "fqlpop_read_probe": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_double)]),
    "fqlpop_envmodel_param_count": (ctypes.c_int, [ctypes.POINTER(EnvModelConfig), ctypes.POINTER(ctypes.c_int64),
                                                   ctypes.POINTER(ctypes.c_int64)]),
    "fqlpop_set_env_model": (ctypes.c_int, [_P, ctypes.POINTER(EnvModelConfig), _F, ctypes.c_int64, _F,
                                            ctypes.c_int64]),
    "fqlpop_rollout": (ctypes.c_int, [_P, _F, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, _F, _F, _F]),
    "fqlpop_envmodel_step": (ctypes.c_int, [_P, _F, _F, ctypes.c_int, _F, _F]),
    "fqlpop_emtrain_param_count": (ctypes.c_int, [ctypes.POINTER(EmTrainConfig), ctypes.POINTER(ctypes.c_int64)]),
    "fqlpop_emtrain_create": (ctypes.c_int, [ctypes.POINTER(EmTrainConfig), _F, ctypes.c_int64, ctypes.c_int,
                                             ctypes.POINTER(_P)]),
    "fqlpop_emtrain_destroy": (ctypes.c_int, [_P]),
    "fqlpop_emtrain_set_frozen_termination": (ctypes.c_int, [_P, _F, ctypes.c_int64]),
    "fqlpop_emtrain_set_dataset": (ctypes.c_int, [_P, _F, _F, _F, _F, ctypes.c_int64]),
    "fqlpop_emtrain_step": (ctypes.c_int, [_P, ctypes.c_int]),
    "fqlpop_emtrain_step_injected": (ctypes.c_int, [_P, _F, _F, _F, _F, _U8]),
    "fqlpop_emtrain_eval": (ctypes.c_int, [_P, _F, _F, _F, _F, _F]),
    "fqlpop_emtrain_read_logs": (ctypes.c_int, [_P, _F]),
    "fqlpop_emtrain_get_params": (ctypes.c_int, [_P, ctypes.c_int, _F, ctypes.c_int64]),
    "fqlpop_emtrain_get_count": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "fqlpop_emtrain_sync": (ctypes.c_int, [_P]),
}
EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libfqlpop.so (no fallback: raises if it is missing)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("FQLPOP_LIB") or LIB_PATH  # FQLPOP_LIB: A/B builds (developer)
    if not os.path.exists(p):
        raise FqlpopError(
            f"{p} not found: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load_library().fqlpop_last_error().decode(errors="replace")
        raise FqlpopError(f"fqlpop error {rc}: {msg}")


def set_engine_option(name: str, value: int) -> None:
    """Process-wide engine option for later Population handles (fqlpop_set_engine_option:
    alternate code paths / stream schedules with the same results; tests and profiling)."""
    check(load_library().fqlpop_set_engine_option(name.encode(), int(value)))


def get_engine_option(name: str) -> int:
    v = ctypes.c_int()
    check(load_library().fqlpop_get_engine_option(name.encode(), ctypes.byref(v)))
    return v.value


def reset_engine_options() -> None:
    check(load_library().fqlpop_reset_engine_options())


def step_streams() -> int:
    """Parallel branches (streams) a population created now would capture its step on
    (fqlpop_step_streams; no GPU call)."""
    v = ctypes.c_int()
    check(load_library().fqlpop_step_streams(ctypes.byref(v)))
    return v.value


def hw_queues_from_env() -> int | None:
    """GPU_MAX_HW_QUEUES, the HIP runtime's hardware queues per process, if the caller set
    it (None otherwise): Population passes it to the engine (option hw_queues), which
    captures the step on one stream below 4."""
    v = os.environ.get("GPU_MAX_HW_QUEUES")
    try:
        return max(1, min(1024, int(v))) if v else None
    except ValueError:
        return None


def is_diagnostic_build() -> bool:
    return bool(load_library().fqlpop_diagnostic_build())


def fptr(a):
    """float32 C-contiguous numpy array -> float* (the array must stay alive)."""
    return a.ctypes.data_as(_F)
