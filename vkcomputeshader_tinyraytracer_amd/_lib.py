"""ctypes binding of the product library libtrt.so (include/trt/abi.h).

There is no fallback: if the in-tree HIP library is missing or fails to load, every entry
point raises.  The CPU oracle under oracle/ is test infrastructure and is never imported
from here.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

from .types import BandLayout, BandXfer, Params, Stats

_HERE = Path(__file__).resolve().parent
# TRT_LIB may point at an experimental build of the same library (tools/build_variants.sh).
LIB_PATH = Path(os.environ["TRT_LIB"]) if os.environ.get("TRT_LIB") else _HERE / "libtrt.so"

_lib: ctypes.CDLL | None = None


class TrtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"trt error {code}: {msg}")
        self.code = code


def raise_hw_queues() -> None:
    """GPU_MAX_HW_QUEUES=32 when it is unset or at HIP's default (<= 4) and the operator did
    not opt out (TRT_KEEP_HW_QUEUES=1).  Only effective before HIP initialises."""
    if os.environ.get("TRT_KEEP_HW_QUEUES", "0") not in ("", "0"):
        return
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    except ValueError:
        return
    if cur <= 4:
        os.environ["GPU_MAX_HW_QUEUES"] = "32"


def lib() -> ctypes.CDLL:
    """Loads libtrt.so (built by __graft_entry__.build() / `make -C .../csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback"
        )
    # PyTorch-ROCm bundles its own HIP runtime (ROCm 7.0) while libtrt.so is linked against
    # /opt/rocm's (7.2, same SONAME).  Measured on the box: when libtrt has initialised HIP
    # before torch is imported, torch's device init fails ("No HIP GPUs are available"); with
    # torch imported first both work.  So when torch is importable it is loaded first.
    # Frames in flight run on their own HIP streams: 32 hardware queues when the environment
    # leaves HIP at its default of 4 (or less), set once here, before torch or libtrt
    # initialises HIP.  TRT_KEEP_HW_QUEUES=1 leaves an operator's setting alone.
    raise_hw_queues()
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(os.fspath(LIB_PATH))
    c_int, c_u32, vp = ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p
    f3 = ctypes.POINTER(ctypes.c_float)
    sigs = {
        "trt_version": (ctypes.c_char_p, []),
        "trt_create": (c_int, [ctypes.POINTER(vp), c_int]),
        "trt_destroy": (c_int, [vp]),
        "trt_last_error": (ctypes.c_char_p, [vp]),
        "trt_set_stream": (c_int, [vp, vp]),
        "trt_upload_scene": (c_int, [vp, vp, vp, c_u32, vp, c_u32, vp, c_u32, c_u32]),
        "trt_update_ubo": (c_int, [vp, vp]),
        "trt_render": (c_int, [vp, ctypes.POINTER(Params), vp, vp, ctypes.POINTER(Stats)]),
        "trt_set_frames_in_flight": (c_int, [vp, c_u32]),
        "trt_set_subtree_split": (c_int, [vp, c_int]),
        "trt_set_deferred_shadows": (c_int, [vp, c_int]),
        "trt_defer_stats": (c_int, [vp, c_u32, ctypes.POINTER(ctypes.c_uint64)]),
        "trt_render_frames": (c_int, [vp, ctypes.POINTER(Params), vp, c_u32, vp, ctypes.c_size_t, c_u32]),
        "trt_frame_times": (c_int, [vp, ctypes.POINTER(ctypes.c_float), c_u32]),
        "trt_timed_launches": (c_u32, [vp, ctypes.POINTER(c_u32), c_u32]),
        "trt_set_frame_batch": (c_int, [vp, c_u32]),
        "trt_synchronize": (c_int, [vp]),
        "trt_output_rows": (c_u32, [ctypes.POINTER(Params)]),
        "trt_params_default": (None, [ctypes.POINTER(Params)]),
        "trt_scene_create": (c_int, [ctypes.POINTER(vp)]),
        "trt_scene_destroy": (None, [vp]),
        "trt_scene_last_error": (ctypes.c_char_p, [vp]),
        "trt_scene_set_batch_size": (c_int, [vp, c_u32]),
        "trt_scene_add_mesh": (c_int, [vp, vp, c_u32, vp, c_u32, vp, f3, f3, f3, c_int]),
        "trt_scene_add_obj": (c_int, [vp, ctypes.c_char_p, vp, f3, f3, f3, c_int]),
        "trt_scene_triangle_count": (c_u32, [vp]),
        "trt_scene_model_count": (c_u32, [vp]),
        "trt_scene_triangles": (vp, [vp]),
        "trt_scene_models": (vp, [vp]),
        "trt_jpeg_create": (c_int, [ctypes.POINTER(vp)]),
        "trt_jpeg_destroy": (None, [vp]),
        "trt_jpeg_last_error": (ctypes.c_char_p, [vp]),
        "trt_jpeg_parse": (c_int, [vp, vp, ctypes.c_size_t]),
        "trt_jpeg_get_info": (c_int, [vp, vp]),
        "trt_jpeg_coefficients": (vp, [vp, c_u32]),
        "trt_jpeg_quant": (vp, [vp, c_u32]),
        "trt_jpeg_decode": (c_int, [vp, vp, vp, c_u32]),
        "trt_upload_envmap_jpeg": (c_int, [vp, vp, ctypes.c_size_t]),
        "trt_write_ppm": (c_int, [ctypes.c_char_p, vp, c_u32, c_u32]),
        "trt_write_png": (c_int, [ctypes.c_char_p, vp, c_u32, c_u32]),
        "trt_multi_create": (c_int, [ctypes.POINTER(vp), ctypes.POINTER(c_int), c_u32]),
        "trt_multi_unique_id": (c_int, [vp]),
        "trt_multi_create_rank": (c_int, [ctypes.POINTER(vp), c_int, c_u32, c_u32, vp]),
        "trt_multi_destroy": (c_int, [vp]),
        "trt_multi_last_error": (ctypes.c_char_p, [vp]),
        "trt_multi_ranks": (c_u32, [vp]),
        "trt_multi_local_count": (c_u32, [vp]),
        "trt_multi_context": (vp, [vp, c_u32]),
        "trt_multi_set_band_groups": (c_int, [vp, c_u32]),
        "trt_multi_upload_scene": (c_int, [vp, vp, vp, c_u32, vp, c_u32, vp, c_u32, c_u32]),
        "trt_multi_update_ubo": (c_int, [vp, vp]),
        "trt_render_multi": (c_int, [vp, ctypes.POINTER(Params), c_u32, c_int, ctypes.POINTER(vp),
                                     ctypes.POINTER(Stats)]),
        "trt_render_multi_frames": (c_int, [vp, ctypes.POINTER(Params), vp, c_u32, c_u32, c_int, c_u32,
                                            ctypes.POINTER(vp), ctypes.c_size_t]),
        "trt_multi_synchronize": (c_int, [vp]),
        "trt_multi_set_self_gather": (c_int, [vp, c_int]),
        "trt_frame_root": (c_u32, [c_u32, c_u32, c_int]),
        "trt_band_frame_row": (c_u32, [c_u32, c_u32, c_u32, c_u32]),
        "trt_band_plan": (c_int, [c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_int, c_u32,
                                  ctypes.POINTER(BandLayout), ctypes.POINTER(BandXfer), c_u32,
                                  ctypes.POINTER(c_u32)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


# Every symbol include/trt/abi.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = (
    "trt_version",
    "trt_create",
    "trt_destroy",
    "trt_last_error",
    "trt_set_stream",
    "trt_upload_scene",
    "trt_update_ubo",
    "trt_render",
    "trt_set_frames_in_flight",
    "trt_set_subtree_split",
    "trt_set_deferred_shadows",
    "trt_defer_stats",
    "trt_render_frames",
    "trt_frame_times",
    "trt_timed_launches",
    "trt_set_frame_batch",
    "trt_synchronize",
    "trt_output_rows",
    "trt_params_default",
    "trt_scene_create",
    "trt_scene_destroy",
    "trt_scene_last_error",
    "trt_scene_set_batch_size",
    "trt_scene_add_mesh",
    "trt_scene_add_obj",
    "trt_scene_triangle_count",
    "trt_scene_model_count",
    "trt_scene_triangles",
    "trt_scene_models",
    "trt_jpeg_create",
    "trt_jpeg_destroy",
    "trt_jpeg_last_error",
    "trt_jpeg_parse",
    "trt_jpeg_get_info",
    "trt_jpeg_coefficients",
    "trt_jpeg_quant",
    "trt_jpeg_decode",
    "trt_upload_envmap_jpeg",
    "trt_write_ppm",
    "trt_write_png",
    "trt_multi_create",
    "trt_multi_unique_id",
    "trt_multi_create_rank",
    "trt_multi_destroy",
    "trt_multi_last_error",
    "trt_multi_ranks",
    "trt_multi_local_count",
    "trt_multi_context",
    "trt_multi_set_band_groups",
    "trt_multi_upload_scene",
    "trt_multi_update_ubo",
    "trt_render_multi",
    "trt_render_multi_frames",
    "trt_multi_synchronize",
    "trt_multi_set_self_gather",
    "trt_frame_root",
    "trt_band_frame_row",
    "trt_band_plan",
)
