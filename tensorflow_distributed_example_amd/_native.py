"""ctypes bindings for the in-tree native libraries.

``hip()``  -> libtde_hip.so  (gfx950 kernels + RCCL), loaded lazily on first GPU use.
``host()`` -> libtde_host.so (TCP store/RPC, PS, TensorBundle, events, crc32c).

On a machine with a GPU the HIP library is REQUIRED: ``hip()`` raises if it is
missing instead of silently falling back to PyTorch kernels.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the HIP library: shares libamdhip64/librccl)

_LIBDIR = Path(__file__).resolve().parent / "_lib"
_lock = threading.Lock()
_hip = None
_host = None

p = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f32 = C.c_float
sz = C.c_size_t
u32 = C.c_uint32

_HIP_PROTOS = {
    "tde_gemm_pick_splits": (i32, [i32, i32, i32]),
    "tde_gemm_nt_bf16": (i32, [p, i32, p, i32, p, i32, i32, i32, i32, f32, i32, i32, p, i32, p, i32, p]),
    "tde_conv3x3c1_relu_pool_fwd": (i32, [p, p, p, p, p, i32, p, i32, i32, i32, i32, p, i32, p]),
    "tde_conv3x3c1_relu_pool_bwd": (i32, [p, p, p, i32, p, i32, i32, p, p, i32, i32, i32, i32, p]),
    "tde_head_xent": (i32, [p, i32, p, i32, p, p, p, i32, i32, i32, f32, i32, p, p, p, p, i32, p, i32,
                            p, i32, p, p, i32, p, i32, p, p, i32, p]),
    "tde_convnet_fwd": (i32, [p, p, p, p, i32, p, p, i32, p, i32, i32, i32, i32, p, i32, p, i64, i64, p, i32, i64,
                              p]),
    "tde_convnet_bwd": (i32, [p, p, i32, p, p, i32, i64, p, p, p, i32, i32, p, f32, p, p, i32, p, i32, p, p, p, p,
                              p, p, i32, i32, i32, p, p, p, p]),
    "tde_convnet_cgrad_reduce": (i32, [p, i32, p, p, p]),
    "tde_convnet_fwd_f32": (i32, [p, p, p, p, i32, p, p, i32, p, i32, i32, i32, i32, p, p, i64, i64, p, i32, i64,
                                  p]),
    "tde_convnet_bwd_f32": (i32, [p, p, i32, p, p, i32, i64, p, p, p, i32, i32, p, f32, p, p, i32, p, i32, p, p,
                                  p, p, p, p, i32, i32, i32, p, p, p, p, i32, i64, p]),
    "tde_flat_apply": (i32, [p, p, p, p, p, p, i32, f32, f32, f32, f32, f32, p, i32, i32, i64, p, p]),
    "tde_noop": (i32, [i32, i32, p]),
    "tde_cnet_abi_sizes": (i32, [p, i32]),
    "tde_cgen_supported": (i32, [i32, i32]),
    "tde_cgen_fwd": (i32, [i32, i32, p, p, p, p, p, i32, i64, p, i32, p, i32, p, p, p, i32, i32, i32, p]),
    "tde_cgen_bwd": (i32, [i32, i32, p, p, i32, p, p, i32, i64, p, p, p, i32, i32, p, f32, p, p, p, i32, p, p, p,
                           p, p, p, p, p, p, i32, i64, p, p, p, i32, i32, i32, p]),
    "tde_xgmi_abi_sizes": (i32, [p, i32]),
    "tde_optim_table_size": (i32, [p, i32]),
    "tde_optim_build_table": (i32, [p, i32, p]),
    "tde_optim_apply": (i32, [p, p, p, p, p, p, p, i32, p, i32, f32, f32, f32, f32, f32, f32, i32, p, p]),
    "tde_shadow_refresh": (i32, [p, p, p, p, i32, p]),
    # layer-wise kernel library (csrc/kernels/layers.hip)
    "tde_igemm": (i32, [p, i64, i32, p, i64, i32, i32, i32, i32, p, i32, p, i64, i32, f32, p, i64, i32, p, i32,
                        p, p, p, p]),
    "tde_igemm_wgrad_scratch_elems": (i64, [i32, i32, i32]),
    "tde_igemm_tune": (None, [i32, i32, i32, i32, i32, i32]),
    "tde_igemm_tile_min": (None, [i32]),
    "tde_igemm_big_dgrad": (None, [i32]),
    "tde_igemm_wgrad_dma": (None, [i32]),
    "tde_igemm_mfma32": (None, [i32]),
    "tde_layers_deterministic": (None, [i32]),
    "tde_layers_is_deterministic": (i32, []),
    "tde_igemm_mfma32_launches": (C.c_ulonglong, []),
    "tde_igemm_wgrad_tile_cap": (None, [i32]),
    "tde_igemm_wgrad_dma_launches": (C.c_ulonglong, []),
    "tde_igemm_big_launches": (C.c_ulonglong, []),
    "tde_bn_fwd": (i32, [p, p, p, i64, i32, i32, p, p, p, p, f32, p, p, f32, f32, p, i32, f32, C.c_ulonglong,
                         p, i32, i32, p]),
    "tde_bn_bwd": (i32, [p, p, p, i64, i32, i32, p, p, p, i32, f32, C.c_ulonglong, p, i32, i32, p, p, i32, p,
                         i32, p, p, p, i32, p]),
    "tde_igemm_dgrad_bnsum": (i32, [p, p, i32, i32, i32, p, p, i64, i32, p, p]),
    "tde_bnsum_bytes": (i32, []),
    "tde_act_bwd": (i32, [p, p, i64, i32, i32, p, p, p]),
    "tde_maxpool": (i32, [p, p, p, p, p, i32, p, i32, p]),
    "tde_bn_relu_maxpool_fwd": (i32, [p, i64, i32, i32, p, p, p, p, f32, p, p, f32, f32, p, p, p, p, p]),
    "tde_bn_pool_bwd": (i32, [p, p, p, i64, i32, p, p, p, i32, p, p, i32, p, p, p, p, p]),
    "tde_gap": (i32, [p, p, i32, i32, i32, i32, i32, p]),
    "tde_pad": (i32, [p, p, p, i32, i32, p]),
    "tde_xent": (i32, [p, i64, p, i32, i32, f32, p, i64, p, p, i32, p, p]),
    "tde_colstats": (i32, [p, i64, i32, p, p]),
    "tde_cast_f32_bf16": (i32, [p, p, i64, p]),
    "tde_smallconv_fwd": (i32, [p, p, p, i32, p, p, p, p]),
    "tde_smallconv_dgrad": (i32, [p, p, p, i32, p, p]),
    "tde_smallconv_ok": (i32, [i32, i32, i32, i32, i32]),
    "tde_smallconv_wgrad": (i32, [p, p, p, p, p]),
    "tde_smallconv_wgrad_ok": (i32, [i32, i32, i32, i32]),
    "tde_im2col": (i32, [p, p, i32, p, p, p, p]),
    # persistent halo-tile 3x3 conv (csrc/kernels/haloconv.hip)
    "tde_halo_conv_ok": (i32, [i32, i32, i32, i32, i32]),
    "tde_halo_stamps": (None, [p]),
    "tde_halo_conv3x3": (i32, [p, p, i64, i64, i32, p, i32, p, i32, i32, i32, i32, p]),
    "tde_halo_wgrad_ok": (i32, [i32, i32, i32, i32, i32]),
    "tde_halo_wgrad_mfma": (None, [i32]),
    "tde_stem_wgrad_ok": (i32, [i32, i32, i32, i32, i32, i32, i32, i32, i32, i32]),
    "tde_stem_wgrad_scratch_elems": (i64, [i32, i32, i32]),
    "tde_stem_wgrad": (i32, [p, p, p, p, i64, i32, i32, i32, i32, i32, i32, i32, p]),
    "tde_stem_fwd_ok": (i32, [i32, i32, i32, i32, i32, i32, i32, i32, i32, i32]),
    "tde_stem_fwd": (i32, [p, p, p, p, i32, i32, i32, i32, i32, i32, i32, p]),
    "tde_halo_wgrad_scratch_elems": (i64, [i32, i32, i32]),
    "tde_halo_wgrad3x3": (i32, [p, p, p, p, i64, i32, i32, i32, p]),
    "tde_splitk_reduce": (i32, [p, i32, i64, p, p]),
    "tde_stem_pack": (i32, [p, p, p, p, p, p]),
    "tde_gather_rows_dev": (i32, [p, i64, i64, p, i64, p, p, p]),
    "tde_copy_pairs": (i32, [i32, p, p, p, p]),
    "tde_smallnet_limits": (i32, [p]),
    "tde_smallnet_step": (i32, [p, i32, i32, i32, p, p, i32, i32, i32, p, p, p, i32, p, i32, p, p, f32, p, i32,
                                p, p]),
    "tde_smallnet_wgrad": (i32, [p, i32, p, i32, i32, i32, p, i32, p, i32, p, p, p, p, p, p, i32, i32, f32, f32,
                                 f32, f32, f32, p]),
    "tde_dgrad_phase_zero": (i32, [p, p, C.c_uint, p]),
    "tde_stem_unpack_wgrad": (i32, [p, p, p, p]),
    # RCCL
    "tde_nccl_version": (i32, []),
    "tde_nccl_error_string": (C.c_char_p, [i32]),
    "tde_nccl_get_unique_id": (i32, [C.c_char_p]),
    "tde_nccl_unique_id_bytes": (i32, []),
    "tde_nccl_comm_init_rank": (i32, [C.POINTER(p), i32, C.c_char_p, i32, i32]),
    "tde_nccl_comm_init_ranks_grouped": (i32, [C.POINTER(p), i32, C.c_char_p, i32, C.POINTER(i32), i32]),
    "tde_nccl_comm_init_all": (i32, [C.POINTER(p), i32, C.POINTER(i32)]),
    "tde_nccl_comm_destroy": (i32, [p]),
    "tde_nccl_comm_abort": (i32, [p]),
    "tde_nccl_comm_async_error": (i32, [p]),
    "tde_nccl_group_start": (i32, []),
    "tde_nccl_group_end": (i32, []),
    "tde_nccl_all_reduce": (i32, [p, p, sz, i32, i32, p, p]),
    "tde_nccl_broadcast": (i32, [p, p, sz, i32, i32, p, p]),
    "tde_nccl_all_gather": (i32, [p, p, sz, i32, p, p]),
    "tde_nccl_reduce_scatter": (i32, [p, p, sz, i32, i32, p, p]),
    "tde_nccl_send": (i32, [p, sz, i32, i32, p, p]),
    "tde_nccl_recv": (i32, [p, sz, i32, i32, p, p]),
    # single-node xGMI peer-memory all-reduce (csrc/comm/xgmi_allreduce.hip)
    "tde_xgmi_window_bytes": (sz, [i64]),
    "tde_xgmi_max_ranks": (i32, []),
    "tde_xgmi_max_blocks": (i32, []),
    "tde_xgmi_ipc_handle_bytes": (i32, []),
    "tde_xgmi_alloc": (i32, [i32, i64, i32, C.POINTER(p), C.POINTER(p), C.POINTER(p), C.c_char_p]),
    "tde_xgmi_open": (i32, [i32, C.c_char_p, C.POINTER(p)]),
    "tde_xgmi_close": (i32, [p]),
    "tde_enable_peer_access": (i32, [i32, i32]),
    "tde_xgmi_free": (i32, [p, p, p]),
    "tde_xgmi_error": (i32, [p]),
    "tde_xgmi_epoch": (i64, [p]),
    "tde_xgmi_trace_words": (i32, []),
    "tde_xgmi_push_spec": (i32, [i64, i64, p, p, i32, i32, i32, i64, p]),
    "tde_xgmi_set_trace": (i32, [p, p, i32]),
    "tde_xgmi_set_wide": (i32, [i32]),
    "tde_xgmi_threads": (i32, [i32, i32]),
    "tde_xgmi_all_reduce": (i32, [p, i64, i64, p, p, p, i32, i32, i32, i32, i64, p]),
    "tde_xgmi_all_reduce_apply": (i32, [p, i64, i64, p, p, p, i32, i32, i32, i32, i64, p, p]),
    "tde_xgmi_all_reduce_group": (i32, [i32, p, i64, i64, p, p, p, i32, i32, i32, i32, i64, p, p]),
}

_EXTRA_HIP_PROTOS: dict = {}
_HOST_PROTOS: dict = {
    "tde_crc32c": (u32, [p, sz]),
    "tde_crc32c_extend": (u32, [u32, p, sz]),
    "tde_crc32c_masked": (u32, [p, sz]),
    "tde_crc32c_mask": (u32, [u32]),
    "tde_crc32c_unmask": (u32, [u32]),
    # tf.data pipeline engine (csrc/data/pipeline.cpp)
    "tde_shuffle_new": (p, [i64, C.c_ulonglong]),
    "tde_shuffle_free": (None, [p]),
    "tde_shuffle_feed": (i64, [p, p, i64, p]),
    "tde_shuffle_drain": (i64, [p, p]),
    "tde_shuffle_size": (i64, [p]),
    "tde_gather_rows": (i32, [p, i64, i64, p, i64, p, i32]),
}


def register_hip(protos: dict):
    """Add prototypes (used by kernel modules defined in other files)."""
    _EXTRA_HIP_PROTOS.update(protos)
    if _hip is not None:
        _apply(_hip, protos)


def register_host(protos: dict):
    _HOST_PROTOS.update(protos)
    if _host is not None:
        _apply(_host, protos)


def _apply(lib, protos):
    for name, (res, args) in protos.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def lib_path(name: str) -> Path:
    return _LIBDIR / name


def hip_available() -> bool:
    return lib_path("libtde_hip.so").exists()


def hip():
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                # TDE_HIP_LIB: another in-tree build of the kernel library (A/B timing of kernel variants)
                path = lib_path(os.environ.get("TDE_HIP_LIB", "libtde_hip.so"))
                if not path.exists():
                    raise RuntimeError(
                        f"native HIP library missing: {path}. Build it with "
                        "`python -m tensorflow_distributed_example_amd._build` (hipcc, gfx950).")
                lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
                _apply(lib, _HIP_PROTOS)
                _apply(lib, _EXTRA_HIP_PROTOS)
                _hip = lib
    return _hip


def host():
    global _host
    if _host is None:
        with _lock:
            if _host is None:
                path = lib_path("libtde_host.so")
                if not path.exists():
                    from . import _build
                    _build.build_host()
                lib = C.CDLL(str(path))
                _apply(lib, _HOST_PROTOS)
                _host = lib
    return _host


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def native_loaded() -> dict:
    return {"hip": _hip is not None, "host": _host is not None}


os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
