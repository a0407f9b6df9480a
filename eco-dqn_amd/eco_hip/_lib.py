"""ctypes binding of libecohip.so (include/eco_hip.h).

The library is the product: there is no CPU or PyTorch fallback.  If the shared
object is missing this module raises ImportError; if a call fails the error is
raised as the exception type the reference raises for the same condition.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ECO_HIP_LIB", os.path.join(_HERE, "libecohip.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libecohip.so not found at {LIB_PATH}: build it with `make -C eco-dqn_amd` "
                      "(hipcc --offload-arch=gfx950); eco_hip has no fallback path")
lib = ctypes.CDLL(LIB_PATH)

# ---- status codes / enums (eco_hip.h) ----
ECO_OK, ECO_ERR_ARG, ECO_ERR_HIP, ECO_ERR_PAST_END, ECO_ERR_BASIS, ECO_ERR_TARGET, ECO_ERR_OBSERVABLE, \
    ECO_ERR_GRAPH, ECO_ERR_KEY, ECO_ERR_INDEX = range(10)
ECO_MAX_OBS = 16          # observables per env (MAIN_OBSERVABLES has 13)
ECO_MPNN_MAX_OBS = 16     # MPNN n_obs_in limit (node-feature rows of obs_x_stride(n_obs_in) floats)
ECO_ENV_SCALARS = 16
ECO_TARGET_CUT, ECO_TARGET_ENERGY, ECO_TARGET_MIN_COVER, ECO_TARGET_MIN_CUT, ECO_TARGET_MAX_IND_SET, \
    ECO_TARGET_MAX_CLIQUE, ECO_TARGET_MIN_DOM_SET = range(1, 8)


def obs_x_stride(n_obs):
    """ECO_OBS_X_STRIDE: floats per node-feature row of obs_x."""
    return 8 if n_obs <= 8 else 16
ECO_MAX_SPINS = 2048
ECO_COMPACT_MAX_SPINS = 8192  # include/eco_hip.h: compact replay (sample rebuilds s' in LDS)
ECO_NORM_PER_GRAPH, ECO_NORM_PER_CALL, ECO_NORM_PER_CALL_REUSE = 0, 1, 2
ECO_GRAPH_ER, ECO_GRAPH_BA = 1, 2
# kernel-path policy bits (eco_set_kernel_paths)
ECO_PATH_NO_DENSE, ECO_PATH_NO_DL, ECO_PATH_NO_SHARED, ECO_PATH_NO_PAIR, ECO_PATH_DENSE2_FWD = 1, 2, 4, 8, 16


class EnvConfig(ctypes.Structure):
    _fields_ = [("n_spins", ctypes.c_int32), ("max_steps", ctypes.c_int32), ("n_obs", ctypes.c_int32),
                ("obs_ids", ctypes.c_int32 * ECO_MAX_OBS), ("reward_signal", ctypes.c_int32),
                ("norm_rewards", ctypes.c_int32), ("reversible_spins", ctypes.c_int32),
                ("spin_basis", ctypes.c_int32), ("stopping", ctypes.c_int32),
                ("has_basin_reward", ctypes.c_int32), ("has_stag_punishment", ctypes.c_int32),
                ("horizon_length", ctypes.c_int32), ("optimisation_target", ctypes.c_int32),
                ("basin_reward", ctypes.c_double),
                ("stag_punishment", ctypes.c_double)]


class GraphSet(ctypes.Structure):
    _fields_ = [("n_graphs", ctypes.c_int32), ("n_spins", ctypes.c_int32), ("row_ptr", ctypes.c_void_p),
                ("edge_base", ctypes.c_void_p), ("edges", ctypes.c_void_p), ("deg", ctypes.c_void_p),
                ("max_deg", ctypes.c_void_p), ("meta", ctypes.c_void_p), ("valid", ctypes.c_void_p),
                ("unit_weights", ctypes.c_int32), ("adjbits", ctypes.c_void_p)]


class Replay(ctypes.Structure):
    _fields_ = [("capacity", ctypes.c_int32), ("n_spins", ctypes.c_int32), ("x_stride", ctypes.c_int32),
                ("xs", ctypes.c_void_p),
                ("xn", ctypes.c_void_p), ("gid", ctypes.c_void_p), ("act", ctypes.c_void_p),
                ("rew", ctypes.c_void_p), ("done", ctypes.c_void_p)]


class ActConfig(ctypes.Structure):
    _fields_ = [("epsilon", ctypes.c_float), ("reversible", ctypes.c_int32), ("allowed_value", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("counter", ctypes.c_uint64)]


_P = ctypes.c_void_p
_I = ctypes.c_int32
_SIG = {
    "eco_graphs_prepare": (ctypes.c_int, [ctypes.POINTER(GraphSet), _P]),
    "eco_graphs_adjbits_bytes": (ctypes.c_size_t, [_I, _I]),
    "eco_graphs_generate_workspace_bytes": (ctypes.c_size_t, [_I, _I]),
    "eco_graphs_generate": (ctypes.c_int, [ctypes.POINTER(GraphSet), _I, _I, _I, ctypes.c_double, _I,
                                           ctypes.c_uint64, ctypes.c_int64, _P, _P]),
    "eco_env_state_bytes": (ctypes.c_size_t, [ctypes.POINTER(EnvConfig), _I]),
    "eco_env_reset": (ctypes.c_int, [ctypes.POINTER(EnvConfig), ctypes.POINTER(GraphSet), _P, _I, _P, _P, _P,
                                     ctypes.c_uint64, _P, _P, _P]),
    "eco_env_step": (ctypes.c_int, [ctypes.POINTER(EnvConfig), ctypes.POINTER(GraphSet), _P, _I, _P, _P, _P, _P,
                                    _P, _P]),
    "eco_env_read": (ctypes.c_int, [ctypes.POINTER(EnvConfig), _P, _I, _P, _P, _P, _P]),
    "eco_check_errors": (ctypes.c_int, [_P]),
    "eco_error_word_copy": (ctypes.c_int, [_P, _P]),
    "eco_set_kernel_paths": (_I, [_I]),
    "eco_probe_split2_mfma": (ctypes.c_int, [_P, _P, _P, _I, _I, _P, _P]),
    "eco_env_greedy_actions": (ctypes.c_int, [ctypes.POINTER(EnvConfig), ctypes.POINTER(GraphSet), _P, _I, _P,
                                              _P]),
    "eco_mpnn_param_count": (ctypes.c_size_t, [_I]),
    "eco_mpnn_packed_count": (ctypes.c_size_t, []),
    "eco_mpnn_pack": (ctypes.c_int, [_P, _I, _P, _P]),
    "eco_mpnn_workspace_bytes": (ctypes.c_size_t, [_I, _I]),
    "eco_mpnn_forward": (ctypes.c_int, [_P, _I, ctypes.POINTER(GraphSet), _P, _I, _P, _I, _P,
                                        ctypes.POINTER(ActConfig), _P, _P, _P, _P]),
    "eco_mpnn_forward_pair": (ctypes.c_int, [_P, _P, _I, ctypes.POINTER(GraphSet), _P, _I, _P, _I, _P,
                                             ctypes.POINTER(ActConfig), _P, _P, ctypes.POINTER(ActConfig), _P, _P,
                                             _P]),
    "eco_mpnn_saved_bytes": (ctypes.c_size_t, [_I, _I]),
    "eco_mpnn_backward_workspace_bytes": (ctypes.c_size_t, [_I, _I]),
    "eco_mpnn_backward": (ctypes.c_int, [_P, _I, ctypes.POINTER(GraphSet), _P, _I, _P, _P, _P, _P, _P, _P]),
    "eco_dqn_td": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I, _I, ctypes.c_float, _I, _P, _P, _P, _P]),
    "eco_adam": (ctypes.c_int, [_P, _P, _P, _P, _I, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int64, _P]),
    "eco_replay_push": (ctypes.c_int, [ctypes.POINTER(Replay), _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "eco_replay_sample": (ctypes.c_int, [ctypes.POINTER(Replay), _I, _I, ctypes.c_uint64, ctypes.c_uint64, _P, _P,
                                         _P, _P, _P, _P, _P]),
    "eco_replay_compact_bytes": (ctypes.c_size_t, [_I, _I, _I]),
    "eco_replay_compact_snapshot": (ctypes.c_int, [ctypes.POINTER(EnvConfig), _P, _I, _P, _I, ctypes.c_int64, _P,
                                                   _P]),
    "eco_replay_compact_push": (ctypes.c_int, [ctypes.POINTER(EnvConfig), _P, _I, _P, _I, ctypes.c_int64, _P, _P, _P,
                                               _P]),
    "eco_replay_compact_sample": (ctypes.c_int, [ctypes.POINTER(EnvConfig), _P, ctypes.POINTER(GraphSet), _I, _P, _I,
                                                 _I, ctypes.c_int64, _I, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P, _P, _P, _P,
                                                 _P]),
    "eco_per_create": (_P, [_I, ctypes.c_double, ctypes.c_double]),
    "eco_per_destroy": (None, [_P]),
    "eco_per_len": (_I, [_P]),
    "eco_per_beta": (ctypes.c_double, [_P]),
    "eco_per_full": (ctypes.c_int, [_P]),
    "eco_per_configure_beta_anneal_time": (ctypes.c_int, [_P, ctypes.c_double]),
    "eco_per_add": (ctypes.c_int, [_P, _I, _P]),
    "eco_per_update_priorities": (ctypes.c_int, [_P, _I, _P, _P]),
    "eco_per_rebalance": (ctypes.c_int, [_P]),
    "eco_per_sample": (ctypes.c_int, [_P, _I, _P, ctypes.c_uint64, _P, _P, _P]),
    "eco_per_sample_begin": (ctypes.c_int, [_P, _I, _P]),
    "eco_per_sample_finish": (ctypes.c_int, [_P, _I, _P, ctypes.c_uint64, _P, _P, _P]),
    "eco_per_heap": (ctypes.c_int, [_P, _P, _P]),
    "eco_per_partitions": (_I, [_P, _P, _P]),
    "eco_replay_gather": (ctypes.c_int, [ctypes.POINTER(Replay), _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "eco_last_error": (ctypes.c_char_p, []),
}
for _name, (_res, _args) in _SIG.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTS = sorted(_SIG)


def last_error():
    return lib.eco_last_error().decode()


def check(rc):
    """Map an ABI status code to the reference's exception types."""
    if rc == ECO_OK:
        return
    msg = last_error()
    if rc == ECO_ERR_PAST_END or rc == ECO_ERR_TARGET:
        raise NotImplementedError(msg)
    if rc == ECO_ERR_OBSERVABLE:
        raise AssertionError(msg)
    if rc == ECO_ERR_BASIS:
        raise Exception(msg)
    if rc == ECO_ERR_HIP:
        raise RuntimeError(msg)
    if rc == ECO_ERR_KEY:
        raise KeyError(msg)
    if rc == ECO_ERR_INDEX:
        raise IndexError(msg)
    raise ValueError(msg)


def ptr(t):
    """Raw device pointer of a tensor (None stays NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class kernel_paths:
    """Context manager routing MPNN calls to another product kernel family (eco_set_kernel_paths, ECO_PATH_*
    bits) and restoring the previous policy on exit: `with kernel_paths(ECO_PATH_NO_DENSE): ...`."""

    def __init__(self, mask):
        self.mask = int(mask)

    def __enter__(self):
        self.prev = lib.eco_set_kernel_paths(self.mask)
        return self

    def __exit__(self, *exc):
        lib.eco_set_kernel_paths(self.prev)
        return False
