"""ctypes binding of libskgehip.so (declared in include/skge_hip.h).

torch is imported first on purpose: libskgehip.so needs libamdhip64.so.7 and
torch has already loaded its own copy under that SONAME, so the library binds
to torch's HIP runtime and device pointers / streams are shared.  There is no
CPU fallback: if the library or a GPU is missing, calls raise.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# SKGE_LIB_PATH overrides the library (timing-only ablation builds, tools/ablate.sh)
LIB_PATH = os.environ.get("SKGE_LIB_PATH") or os.path.join(_HERE, "libskgehip.so")

SKGE_TRANSE_L1, SKGE_TRANSE_L2, SKGE_HOLE, SKGE_RESCAL = 0, 1, 2, 3
SKGE_AF_LINEAR, SKGE_AF_SIGMOID, SKGE_AF_TANH, SKGE_AF_RELU = 0, 1, 2, 3
SKGE_SGD, SKGE_ADAGRAD = 0, 1
SKGE_POST_NONE, SKGE_POST_NORMALIZE, SKGE_POST_NORMLESS1 = 0, 1, 2
SKGE_ACC_F32, SKGE_ACC_I16X4, SKGE_ACC_I32X2, SKGE_ACC_FX64, SKGE_ACC_I8X4 = 0, 1, 2, 3, 4

c_p = ctypes.c_void_p
c_i = ctypes.c_int
c_f = ctypes.c_float
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_sz = ctypes.c_size_t


class SkgeTable(ctypes.Structure):
    """Mirror of skge_table_t."""
    _fields_ = [("param", c_p), ("state", c_p), ("acc_sum", c_p), ("acc_cnt", c_p),
                ("acc_touched", c_p), ("rows", c_i), ("width", c_i), ("touched_cap", c_i),
                ("acc_mode", c_i), ("acc_replicas", c_i), ("opt", c_i), ("post", c_i), ("lr", c_f), ("rin", c_f), ("rout", c_f),
                ("fixed_div", c_f), ("gate", c_p), ("upd_count", c_p),
                ("violations", c_p)]


T_P = ctypes.POINTER(SkgeTable)

# name -> (restype, argtypes); the exact set declared in include/skge_hip.h
SIGNATURES = {
    "skge_abi_version": (c_i, []),
    "skge_last_error": (ctypes.c_char_p, []),
    "skge_pair_grad": (c_i, [c_p, c_i, c_i, T_P, T_P, c_i, c_p, c_p, c_i, c_f, c_p, c_p, c_p, c_p]),
    "skge_triple_grad": (c_i, [c_p, c_i, T_P, T_P, c_i, c_p, c_p, c_i, c_p, c_p, c_p]),
    "skge_rescal_wgrad": (c_i, [c_p, T_P, T_P, c_i, c_p, c_p, c_i, c_p, c_p, c_i]),
    "skge_collect_workspace_bytes": (c_sz, [c_i]),
    "skge_accum_collect": (c_i, [c_p, T_P, c_p, c_p, c_p, c_p, c_sz]),
    "skge_accum_reset": (c_i, [c_p, T_P, c_i]),
    "skge_triple_set_bytes": (c_sz, [c_i64]),
    "skge_update_rows": (c_i, [c_p, T_P, c_p, c_p, c_i]),
    "skge_accum_apply": (c_i, [c_p, T_P, c_i, ctypes.POINTER(c_i)]),
    "skge_device_error": (c_i, [c_p, c_i]),
    "skge_rank_workspace_bytes": (c_sz, [c_i, c_i]),
    "skge_rank": (c_i, [c_p, c_i, c_p, c_p, c_i, c_i, c_p, c_i, c_p, c_i64, c_p, c_sz, c_p]),
    "skge_rank_known_workspace_bytes": (c_sz, [c_i, c_i]),
    "skge_rank_known": (c_i, [c_p, c_i, c_p, c_p, c_i, c_i, c_p, c_i, c_p, c_p, c_p, c_p, c_p,
                              c_sz, c_p]),
    "skge_pair_step_workspace_bytes": (c_sz, [c_i, c_i, c_i, c_i]),
    "skge_triple_step_workspace_bytes": (c_sz, [c_i, c_i, c_i, c_i]),
    "skge_triple_step": (c_i, [c_p, c_i, T_P, T_P, c_i, c_p, c_p, c_i, c_p, c_sz, c_p]),
    "skge_pair_step": (c_i, [c_p, c_i, c_i, T_P, T_P, c_i, c_p, c_p, c_i, c_f, c_p, c_sz, c_p]),
    "skge_triple_set_build": (c_i, [c_p, c_p, c_i64, c_p, c_i64]),
    "skge_transe_sample_grad": (c_i, [c_p, c_i, T_P, T_P, c_i, c_p, c_i64, c_p, c_i64, c_i64, c_i,
                                      c_u64, c_p, c_f, c_i, c_p, c_p, c_p]),
    "skge_epoch_permutation": (c_i, [c_p, c_i64, c_u64, c_p, c_p, c_i64]),
    "skge_epoch_advance": (c_i, [c_p, c_p]),
    "skge_runner_create": (c_p, [c_p, c_i, T_P, T_P, c_i, c_p, c_i64, c_p, c_i64, c_i, c_u64, c_p,
                                 c_f, c_i, c_p, c_p]),
    "skge_runner_run": (c_i, [c_p, c_p, c_i]),
    "skge_runner_nlaunches": (c_i, [c_p]),
    "skge_runner_destroy": (None, [c_p]),
    "skge_pair_runner_create": (c_p, [c_p, c_i, c_i, T_P, T_P, c_i, c_p, c_i64, c_p, c_i64, c_i,
                                      c_u64, c_p, c_f, c_i, c_p]),
    "skge_pair_runner_run": (c_i, [c_p, c_p, c_i]),
    "skge_epoch_sample": (c_i, [c_p, c_p, c_i64, c_p, c_i64, c_i, c_u64, c_p, c_i, c_p, c_p]),
    "skge_pair_runner_nlaunches": (c_i, [c_p]),
    "skge_pair_runner_destroy": (None, [c_p]),
    "skge_pipe_runner_create": (c_p, [c_p, T_P, T_P, c_i, c_p, c_i64, c_p, c_i64, c_i, c_u64, c_p,
                                      c_f, c_i, c_p]),
    "skge_pipe_runner_create_ex": (c_p, [c_p, T_P, T_P, c_i, c_p, c_i64, c_p, c_i64, c_i, c_u64,
                                         c_p, c_f, c_i, c_p, c_i]),
    "skge_hole_pipe_runner_create": (c_p, [c_p, c_i, T_P, T_P, c_i, c_p, c_i64, c_p, c_i64, c_i,
                                           c_u64, c_p, c_f, c_i, c_p]),
    "skge_pipe_runner_run": (c_i, [c_p, c_p, c_i]),
    "skge_pipe_runner_error": (c_i, [c_p, c_p]),
    "skge_pipe_runner_profile": (c_i, [c_p, c_p, c_p, c_p, c_i, c_i, c_p, c_i64]),
    "skge_pipe_runner_nlaunches": (c_i, [c_p]),
    "skge_pipe_runner_hot_rows": (c_i, [c_p]),
    "skge_pipe_runner_kernel": (c_i, [c_p]),
    "skge_pipe_runner_destroy": (None, [c_p]),
    "skge_shard_route_workspace_bytes": (c_sz, [c_i, c_i]),
    "skge_shard_route": (c_i, [c_p, c_p, c_p, c_i64, c_i, c_i, c_p, c_p, c_p, c_p, c_sz]),
    "skge_shard_route_cap": (c_i, [c_p, c_p, c_p, c_i64, c_i, c_i, c_i, c_p, c_p, c_p, c_sz,
                                   c_p]),
    "skge_shard_gather": (c_i, [c_p, c_p, c_i, c_i, c_p, c_i64, c_p]),
    "skge_shard_contrib_stride": (ctypes.c_longlong, [c_i]),
    "skge_shard_score": (c_i, [c_p, T_P, c_i, c_p, c_p, c_i64, c_i, c_p, c_p, c_f, c_p, c_p]),
    "skge_shard_accum": (c_i, [c_p, T_P, c_i, c_p, c_p, c_i64]),
    "skge_shard_fold_violations": (c_i, [c_p, c_p, c_p]),
    "skge_pipe_runner_nbatches": (c_i, [c_p]),
    "skge_pipe_dp_record_bytes": (c_sz, [c_i]),
    "skge_pipe_runner_dp_begin": (c_i, [c_p, c_p]),
    "skge_pipe_runner_dp_batch": (c_i, [c_p, c_p, c_i, c_i, c_i, c_p, c_i]),
    "skge_pipe_runner_dp_scatter": (c_i, [c_p, c_p, c_i, c_p, c_i, c_i]),
    "skge_pipe_runner_dp_end": (c_i, [c_p, c_p]),
    "skge_roofline_gather": (c_i, [c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i,
                                   ctypes.c_uint32, c_p]),
    "skge_handoff_probe": (c_i, [c_p, c_p, c_i, c_p]),
}

_lib = None


class SkgeError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load and type the library (no GPU needed to load)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SkgeError("libskgehip.so not built (%s): run `make -C scikit-kge_amd` "
                        "or __graft_entry__.build()" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.skge_abi_version() != 2:
        raise SkgeError("ABI version mismatch")
    _lib = lib
    return lib


def lib():
    return load()


def check(rc, what=""):
    if rc != 0:
        msg = lib().skge_last_error()
        raise SkgeError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))


def require_gpu():
    if not torch.cuda.is_available():
        raise SkgeError("skge_amd needs a ROCm GPU (MI355X); no CPU fallback exists")


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return c_p(s.cuda_stream)


def int_array(*vals):
    return (c_i * len(vals))(*vals)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return c_p(t.data_ptr())


def check_device_error(stream_handle, what="device"):
    """Read and reset the apply kernels' error word (skge_device_error) and
    raise on its bits: 2 = a packed row's count passed 32767, 4 = a
    deterministic fixed-point sum wrapped or reached half its range."""
    rc = lib().skge_device_error(stream_handle, 1)
    if rc < 0:
        raise SkgeError("%s: %s" % (what, lib().skge_last_error().decode()))
    if rc & 2:
        raise SkgeError("%s: a row's per-batch count exceeded 32767 (packed sums may have "
                        "wrapped); use force_f32=True" % what)
    if rc & 4:
        raise SkgeError("%s: a deterministic fixed-point (FX64) sum wrapped past its 2^23 "
                        "range (caught at the add) or decoded at or past 2^22 (half of it); use "
                        "more batches or the default float sums" % what)
    return rc
