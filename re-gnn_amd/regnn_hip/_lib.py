"""ctypes binding of libregnn_hip.so (C-ABI declared in include/regnn_hip.h).

There is no CPU fallback: if the library is missing this module raises at import, and every
wrapper refuses non-ROCm tensors. Pointers are passed as integers from ``Tensor.data_ptr()``;
the stream is torch's current HIP stream, so kernels order with surrounding torch work.
"""
import ctypes
import os

import torch

from .build import LIB

if not os.path.exists(LIB):
    raise ImportError(
        f"regnn_hip: native library {LIB} is missing — build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
        "There is no CPU fallback.")

# REGNN_LIB: another build of the same ABI (A/B measurements of kernel variants, tools/ab_lib.sh)
_so = ctypes.CDLL(os.environ.get("REGNN_LIB", LIB))

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F32 = ctypes.c_float

_SIG = {
    "regnn_abi_version": ([], ctypes.c_int),
    "regnn_gemm_x6_work_floats": ([I64, I64, I32], I64),
    "regnn_copy2d_many": ([P, I32, P], ctypes.c_int),
    "regnn_wide_ln_fwd": ([I64, I32, P, P, P, P, P, P, P, I32, F32, P, P, P, P, P], ctypes.c_int),
    "regnn_wide_ln_slab_rows": ([I64, I32], I64),
    "regnn_wide_ln_bwd": ([I64, I32, P, P, P, P, P, P, P, I32, F32, P, P, P, P, P], ctypes.c_int),
    "regnn_gemm_x6": ([I32, I32, I64, I64, I64, P, I64, P, I64, P, I64, F32, P, I32, P, P, P],
                      ctypes.c_int),
    "regnn_slab_rows": ([I64, I32], I64),
    "regnn_tune": ([I32, I64], I64),
    "regnn_degree": ([P, P, P, I64, F32, I32, P, I32, P, I32, P, P, P], ctypes.c_int),
    "regnn_degree_bwd": ([P, P, P, P, I64, F32, I32, I32, P, I32, P, P, P], ctypes.c_int),
    "regnn_spmm_fwd": ([P, P, P, P, P, P, P, P, P, P, I64, I32, I32, I32, I32, P, I32, P, P, I32,
                        P, P, I32, P, P], ctypes.c_int),
    "regnn_spmm_bwd": ([P, P, P, P, P, P, P, P, P, P, P, P, I32, P, P, I64, I32, I32, I32, I32, P,
                        I32, P, P, I32, P, P, I32, P, P], ctypes.c_int),
    "regnn_spmm_fwd_dropout": ([P, P, P, P, P, P, P, P, P, P, I64, I32, I32, I32, I32, P, I32, P,
                                P, I32, P, P, I32, P, P, ctypes.c_uint32, F32, P], ctypes.c_int),
    "regnn_spmm_bwd_dropout": ([P, P, P, P, P, P, P, P, P, P, P, P, I32, P, P, I64, I32, I32, I32,
                                I32, P, I32, P, P, I32, P, P, I32, P, P, ctypes.c_uint32, F32, P],
                               ctypes.c_int),
    "regnn_spmm_fwd_next": ([P, P, P, P, P, P, P, P, P, P, I64, I32, I32, I32, I32, P, I32, P, P,
                             I32, P, P, I32, P, P, ctypes.c_uint32, F32, P, P, ctypes.c_uint32,
                             F32, P, P], ctypes.c_int),
    "regnn_spmm_bwd_next": ([P, P, P, P, P, P, P, P, P, P, P, P, I32, P, P, I64, I32, I32, I32,
                             I32, P, I32, P, P, I32, P, P, I32, P, P, ctypes.c_uint32, F32, P, P,
                             P, P], ctypes.c_int),
    "regnn_spmm_fwd_fused": ([P, P, P, P, P, P, P, P, P, P, I64, I32, I32, I32, I32, P, I32, P,
                              P, I32, P, P, I32, P, P, P, P, F32, I32, P], ctypes.c_int),
    "regnn_head_gh_next": ([P, I64, I32, I64, I32, P, P, P, I64, P, P, P, P, P], ctypes.c_int),
    "regnn_head_bwd": ([P, I64, I32, I64, I32, P, P, P, P, I64, P, I32, P], ctypes.c_int),
    "regnn_degree_cnt": ([P, P, I32, I64, F32, P, P, I32, P, P, P, P], ctypes.c_int),
    "regnn_degree_cnt_bwd": ([P, P, P, I64, F32, I32, P, I32, P, P, P], ctypes.c_int),
    "regnn_head_fwd_lse": ([P, I64, I32, P, P, I32, I64, P, I64, P, P, I32, P], ctypes.c_int),
    "regnn_head_bwd_z": ([P, I64, I32, I64, I32, P, P, P, P, I64, P, I32, P, P, F32, P, P, P, P,
                          I32, P], ctypes.c_int),
    "regnn_head_argmax": ([P, I64, I32, P, P, I32, P, P], ctypes.c_int),
    "regnn_gatv2_score_fwd": ([P, P, P, P, P, I64, I32, I32, F32, P, P, P], ctypes.c_int),
    "regnn_gatv2_score_bwd_dst": ([P, P, P, P, P, P, I64, I32, I32, F32, P, P, I32, P, P],
                                  ctypes.c_int),
    "regnn_gatv2_score_bwd_src": ([P, P, P, P, P, P, P, I64, I32, I32, F32, P, P, P],
                                  ctypes.c_int),
    "regnn_edge_softmax_fwd": ([P, P, P, P, P, F32, I64, I32, P, P, P], ctypes.c_int),
    "regnn_edge_softmax_bwd": ([P, P, P, P, I64, I32, P, P, I32, P, P], ctypes.c_int),
    "regnn_gat_scores": ([P, P, P, P, P, P, I64, I32, F32, P, P], ctypes.c_int),
    "regnn_rel_reduce": ([P, I64, I32, P, I32, P], ctypes.c_int),
    "regnn_gat_softmax_fwd": ([P, P, P, P, P, P, I64, I32, F32, P, P, P], ctypes.c_int),
    "regnn_gat_softmax_bwd": ([P, P, P, P, P, P, P, P, I64, I32, F32, P, P, P, I32, P, P],
                              ctypes.c_int),
    "regnn_spmm_heads_fwd": ([P, P, P, P, P, P, I64, I32, I32, I32, P, P], ctypes.c_int),
    "regnn_gat_fused_fwd": ([P, P, P, P, P, P, P, P, P, I64, I32, I32, F32, I32, P, P, P],
                            ctypes.c_int),
    "regnn_gat_attn_lse": ([P, P, P, P, P, P, P, I64, I32, F32, P, P, P], ctypes.c_int),
    "regnn_spmm_heads_bwd": ([P, P, P, P, P, P, P, P, I64, I32, I32, I32, P, P], ctypes.c_int),
    "regnn_segment_sum": ([P, P, P, I64, I32, P, P, P], ctypes.c_int),
    "regnn_col_sum": ([P, I64, I32, P, P], ctypes.c_int),
    "regnn_type_project": ([P, I64, I32, I32, I32, P, P, P, P, ctypes.c_uint32, F32, I64, P, P, P],
                           ctypes.c_int),
    "regnn_linear_wgrad": ([P, I64, I32, I64, P, I32, I32, P, I32, P], ctypes.c_int),
    "regnn_row_scale": ([P, P, P, I64, I32, I32, P, ctypes.c_uint32, F32, P, P, P], ctypes.c_int),
    "regnn_softmax_xent": ([P, I64, I32, I64, P, F32, P, P, P], ctypes.c_int),
    "regnn_attn_dots_fwd": ([P, P, P, I64, I32, I32, P, P, P], ctypes.c_int),
    "regnn_attn_dots_bwd": ([P, P, P, P, P, I64, I32, I32, P, P, I32, P], ctypes.c_int),
    "regnn_head_fwd": ([P, I64, I32, P, P, I32, I64, P, I64, F32, P, P, P, P], ctypes.c_int),
    "regnn_sample_count": ([P, P, I64, I32, P, P], ctypes.c_int),
    "regnn_sample_fill": ([P, P, P, I64, I32, U64, P, P, P, P], ctypes.c_int),
    "regnn_ns_batch": ([P, I64, I32, I32, I32, P, P, P, P, P], ctypes.c_int),
    "regnn_ns_labels": ([P, P, P, I32, I64, P, P], ctypes.c_int),
    "regnn_rel_tab": ([P, P, I32, ctypes.c_float, ctypes.c_float, P, P], ctypes.c_int),
    "regnn_rel_tabs": ([P, P, P, P, I32, ctypes.c_float, ctypes.c_float, P], ctypes.c_int),
    "regnn_softmax_xent_fwd": ([P, P, I32, I32, I64, P, P, P, P], ctypes.c_int),
    "regnn_softmax_xent_bwd": ([P, P, P, P, P, I32, I32, I64, P, P], ctypes.c_int),
    "regnn_ns_xent_fwd": ([P, P, P, P, I32, I32, I64, P, P, P, P, P, P], ctypes.c_int),
    "regnn_xent_bwd_colsum": ([P, P, P, P, P, I32, I32, I64, P, P, P], ctypes.c_int),
    "regnn_ns_hop": ([P, P, P, P, I32, I32, I32, P, P, P, I32, P, P, P, P, P, P, P, P, P, P, P, P,
                      P, P, P, P, P, P, I32, P, P, P, P, I32, P], ctypes.c_int),
    "regnn_ns_hop_typed_sums": ([P, P, P, P, I32, I32, I32, P, P, P, I32, P, P, P, P, P, P, P,
                                 I32, I32, P, P, P, P, P, P], ctypes.c_int),
    "regnn_ns_spmm_bwd": ([P, P, P, P, P, P, P, P, P, I32, I64, I32, P], ctypes.c_int),
    "regnn_ns_csc_hub_work_floats": ([I32], I64),
    "regnn_ns_spmm_bwd_csc": ([P, P, P, P, P, P, P, P, P, I32, P, I32, I64, I32, I32, P, P],
                              ctypes.c_int),
    "regnn_ns_typed_agg": ([P, P, P, P, P, P, P, P, P, P, I32, I32, I64, P, P, I64, I64, P],
                           ctypes.c_int),
    "regnn_ns_typed_agg_bwd": ([P, P, P, P, P, P, P, P, P, I32, I32, I64, P, P, I64, I64, P, I32,
                                I32, P], ctypes.c_int),
    "regnn_ns_spmm_strided_fwd": ([P, P, I32, P, P, P, P, P, P, P, I64, I32, P], ctypes.c_int),
    "regnn_ns_slot_agg": ([P, I32, P, P, P, P, P, I32, I32, I32, I64, P, I64, P], ctypes.c_int),
    "regnn_ns_slot_agg_bwd": ([P, I32, P, P, P, P, P, I64, I32, I32, I32, P, I32, I32, P],
                              ctypes.c_int),
    "regnn_nsm_slab_floats": ([P, I32], I64),
    "regnn_nsm_step": ([P, P, P], ctypes.c_int),
    "regnn_adam_flat": ([P, P, P, P, I64, F32, F32, F32, F32, F32, F32, P, P, P], ctypes.c_int),
    "regnn_typed_gather": ([P, I64, P, P, I32, P, I32, P, P], ctypes.c_int),
    "regnn_typed_scatter": ([P, I64, P, P, I32, P, I32, P, P], ctypes.c_int),
    "regnn_typed_chunks": ([I64, I32, I32], I64),
    "regnn_typed_slab_floats": ([I64, I32, I32, I32], I64),
    "regnn_typed_linear_fwd": ([P, P, P, I64, I32, P, P, P, I32, I32, P, P], ctypes.c_int),
    "regnn_typed_linear_wgrad": ([P, P, P, I64, I32, P, P, I32, I32, I32, P, P, P, P, P],
                                 ctypes.c_int),
}

for _name, (_args, _ret) in _SIG.items():
    if os.environ.get("REGNN_LIB") and not hasattr(_so, _name):
        continue                  # an A/B build of an older tree: calls to it would fail loudly
    _f = getattr(_so, _name)
    _f.argtypes = _args
    _f.restype = _ret

EXPORTED = tuple(_SIG)
ABI_VERSION = 46
# (an A/B build of an older tree through REGNN_LIB may trail the ABI: a timing run only)
if _so.regnn_abi_version() != ABI_VERSION and not os.environ.get("REGNN_LIB"):
    raise ImportError(f"regnn_hip: ABI mismatch ({_so.regnn_abi_version()} != {ABI_VERSION}); "
                      "rebuild the library")

F32_CODE, BF16_CODE = 0, 1
SELF_PRESCALED = 0x100        # or-ed into the dtype of regnn_spmm_bwd* (regnn_hip.h)
_ERR = {1: "invalid argument", 2: "unsupported shape/dtype", 3: "kernel launch failed"}


def dtype_code(t):
    if t.dtype == torch.float32:
        return F32_CODE
    if t.dtype == torch.bfloat16:
        return BF16_CODE
    raise TypeError(f"regnn_hip: unsupported feature dtype {t.dtype} (float32 / bfloat16)")


# Device of a call: every pointer ptr() forms is an int tagged with its tensor's device, so
# call() reads the devices from its own arguments (no state carried between calls: a failure
# while arguments are assembled cannot leak into the next launch). stream() is a placeholder
# that call() replaces with the current stream of the TENSORS' device (not of torch's current
# device), and the launch runs under that device.
class DevPtr(int):
    """Tensor.data_ptr() tagged with the tensor's device index (.dev); passes as a plain int."""

    def __new__(cls, value, dev):
        o = int.__new__(cls, value)
        o.dev = dev
        return o


class _StreamArg:
    """stream() placeholder: call() substitutes the current HIP stream of the call's device."""

    def __repr__(self):
        return "<regnn_hip current stream>"


_STREAM = _StreamArg()


def ptr(t):
    """device pointer of a tensor (None -> NULL); refuses CPU tensors: no CPU fallback."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("regnn_hip kernels need ROCm device tensors (there is no CPU path)")
    return DevPtr(t.data_ptr(), t.device.index)


def stream():
    """the current HIP stream of the call's device, filled in by call()."""
    return _STREAM


def call(name, *args):
    devs = {a.dev for a in args if isinstance(a, DevPtr)}
    if len(devs) > 1:
        raise RuntimeError(f"regnn_hip.{name}: tensors on different devices")
    dev = devs.pop() if devs else None
    if any(a is _STREAM for a in args):
        s = torch.cuda.current_stream(dev).cuda_stream
        args = tuple(s if a is _STREAM else a for a in args)
    if dev is not None and dev != torch.cuda.current_device():
        with torch.cuda.device(dev):
            rc = getattr(_so, name)(*args)
    else:
        rc = getattr(_so, name)(*args)
    if rc != 0:
        raise RuntimeError(f"regnn_hip.{name} failed: {_ERR.get(rc, rc)}")


def slab_rows():
    return int(_so.regnn_slab_rows(0, 0))


def typed_slab_floats(n, T, K, O):
    """fp32 elements of regnn_typed_linear_wgrad's chunk-partial slab."""
    v = int(_so.regnn_typed_slab_floats(int(n), int(T), int(K), int(O)))
    if v < 0:
        raise RuntimeError("regnn_hip.regnn_typed_slab_floats: invalid arguments")
    return max(v, 1)
