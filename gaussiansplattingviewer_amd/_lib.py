"""ctypes binding of libgsr.so, the C ABI declared in include/gsr.h.

This is the only way the package reaches the GPU: there is no CPU or PyTorch fallback.  If
the library is missing or has no HIP device, every entry point raises RuntimeError.
"""
from __future__ import annotations

import atexit
import ctypes
import functools
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# GSR_LIB: another build of the library (A/B builds in tools/ab.sh); default the in-tree libgsr.so
LIB_PATH = os.environ.get("GSR_LIB") or os.path.join(_HERE, "libgsr.so")
ABI_VERSION = 3

GSR_OPT_BLEND_CULL = 1
GSR_OPT_BLEND_FAST = 2
GSR_OPT_DEPTH_SORT = 11
GSR_OPT_TIGHT_BINNING = 13
GSR_OPT_FRAME_GRAPHS = 14
GSR_OPT_SECOND_STREAM = 15

# Symbols include/gsr.h declares (checked by the CPU test suite).
EXPORTED_SYMBOLS = (
    "gsr_abi_version", "gsr_last_error", "gsr_create", "gsr_destroy", "gsr_reserve",
    "gsr_forward", "gsr_get_binning", "gsr_mark_visible", "gsr_depth_argsort",
    "gsr_set_timing", "gsr_stage_times", "gsr_stage_name", "gsr_set_option",
    "gsr_ply_probe", "gsr_ply_load", "gsr_disparity_colors", "gsr_pack_image",
    "gsr_tile_row_pairs", "gsr_frame_graph_stats", "gsr_get_option",
)

GSR_PACK_RGBA_F32 = 0
GSR_PACK_RGB8 = 1
GSR_PACK_R16 = 2


class GsrGaussians(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int64), ("D", ctypes.c_int32), ("M", ctypes.c_int32),
        ("scale_modifier", ctypes.c_float),
        ("means3D", ctypes.c_void_p), ("scales", ctypes.c_void_p),
        ("rotations", ctypes.c_void_p), ("opacities", ctypes.c_void_p),
        ("shs", ctypes.c_void_p), ("colors_precomp", ctypes.c_void_p),
        ("cov3D_precomp", ctypes.c_void_p),
    ]


class GsrRasterSettings(ctypes.Structure):
    _fields_ = [
        ("image_width", ctypes.c_int32), ("image_height", ctypes.c_int32),
        ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
        ("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p),
        ("campos", ctypes.c_void_p), ("bg", ctypes.c_void_p),
        ("tile_row_begin", ctypes.c_int32), ("tile_row_end", ctypes.c_int32),
        ("prefiltered", ctypes.c_int32), ("debug", ctypes.c_int32),
    ]


class GsrOutputs(ctypes.Structure):
    _fields_ = [
        ("color", ctypes.c_void_p), ("radii", ctypes.c_void_p),
        ("depths", ctypes.c_void_p), ("means2D", ctypes.c_void_p),
        ("conic_opacity", ctypes.c_void_p), ("rgb", ctypes.c_void_p),
        ("tiles_touched", ctypes.c_void_p), ("final_T", ctypes.c_void_p),
        ("n_contrib", ctypes.c_void_p), ("num_rendered", ctypes.c_int64),
    ]


class GsrPlyInfo(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int64), ("sh_coeffs", ctypes.c_int32), ("binary", ctypes.c_int32),
        ("bbox_min", ctypes.c_float * 3), ("bbox_max", ctypes.c_float * 3),
        ("center", ctypes.c_float * 3),
    ]


_lock = threading.Lock()
_lib = None
_contexts: dict[int, ctypes.c_void_p] = {}


def _declare(lib: ctypes.CDLL) -> None:
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    lib.gsr_abi_version.restype = i32
    lib.gsr_last_error.restype = ctypes.c_char_p
    lib.gsr_create.argtypes = [ctypes.POINTER(vp)]
    lib.gsr_destroy.argtypes = [vp]
    lib.gsr_destroy.restype = None
    lib.gsr_reserve.argtypes = [vp, i64, i64]
    lib.gsr_forward.argtypes = [vp, ctypes.POINTER(GsrGaussians),
                                ctypes.POINTER(GsrRasterSettings), ctypes.POINTER(GsrOutputs), vp]
    lib.gsr_get_binning.argtypes = [vp, vp, vp, vp, ctypes.POINTER(i64),
                                    ctypes.POINTER(ctypes.c_int32), vp]
    lib.gsr_mark_visible.argtypes = [vp, vp, i64, vp, vp, vp, vp]
    lib.gsr_tile_row_pairs.argtypes = [vp, vp, i32, vp]
    lib.gsr_depth_argsort.argtypes = [vp, vp, i64, ctypes.POINTER(ctypes.c_float), vp, vp, vp]
    lib.gsr_set_timing.argtypes = [vp, i32]
    lib.gsr_stage_times.argtypes = [vp, ctypes.POINTER(ctypes.c_float), i32]
    lib.gsr_stage_name.argtypes = [i32]
    lib.gsr_stage_name.restype = ctypes.c_char_p
    lib.gsr_set_option.argtypes = [vp, i32, i64]
    lib.gsr_get_option.argtypes = [vp, i32, ctypes.POINTER(i64)]
    lib.gsr_frame_graph_stats.argtypes = [vp, ctypes.POINTER(i64), i32]
    lib.gsr_ply_probe.argtypes = [ctypes.c_char_p, ctypes.POINTER(GsrPlyInfo)]
    lib.gsr_ply_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(GsrPlyInfo), vp, vp, vp, vp, vp,
                                 i32, vp]
    lib.gsr_disparity_colors.argtypes = [vp, i64, ctypes.POINTER(ctypes.c_float),
                                         ctypes.POINTER(ctypes.c_float), ctypes.c_float, vp, vp]
    lib.gsr_pack_image.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, vp, vp]
    for name in ("gsr_disparity_colors", "gsr_pack_image", "gsr_create", "gsr_reserve", "gsr_forward", "gsr_get_binning",
                 "gsr_mark_visible", "gsr_depth_argsort", "gsr_set_timing", "gsr_tile_row_pairs",
                 "gsr_stage_times", "gsr_set_option", "gsr_get_option", "gsr_ply_probe", "gsr_ply_load",
                 "gsr_frame_graph_stats"):
        getattr(lib, name).restype = i32


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and return libgsr.so; raise RuntimeError if it is absent or stale."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"libgsr.so not found at {path}: the HIP rasterizer is not built "
                "(run `python -c 'import __graft_entry__ as g; g.build()'` or "
                "`make -C gaussiansplattingviewer_amd/csrc`). There is no CPU fallback.")
        lib = ctypes.CDLL(path)
        _declare(lib)
        ver = lib.gsr_abi_version()
        if ver != ABI_VERSION:
            raise RuntimeError(f"libgsr.so ABI version {ver} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def check(rc: int, what: str) -> int:
    if rc < 0:
        msg = load_library().gsr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")
    return rc


@functools.lru_cache(maxsize=None)
def _native_shares_library() -> bool:
    """The `_native` extension links the in-tree libgsr.so; contexts are shared with it only
    when this module loaded that same file (not a GSR_LIB A/B build).  LIB_PATH is fixed at
    import, so the answer is computed once (the forward asks on every frame)."""
    default = os.path.join(_HERE, "libgsr.so")
    return (os.path.exists(LIB_PATH) and os.path.exists(default) and
            os.path.samefile(LIB_PATH, default))


def context(device_index: int, slot: int = 0) -> ctypes.c_void_p:
    """The process-wide gsr_context of a device (created on first use, on that device).

    `slot` selects one of several independent contexts per device (own workspace, own
    second stream): frames rendered through different slots on different streams may be in
    flight at the same time (`pipeline.FramePipeline`).  Slot 0 is the context the `_C`
    extension (`_native.so`) renders with, so the upstream entry points and this module share
    one workspace and `binning_state()` sees a `GaussianRasterizer` forward (its tight lists
    unless GSR_OPT_TIGHT_BINNING is 0).  Under GSR_LIB (an A/B build) slot 0 is a context of
    that build, and `GaussianRasterizer` renders through it by ctypes instead of `_C`."""
    import torch

    lib = load_library()
    key = (int(device_index), int(slot))
    with _lock:
        ctx = _contexts.get(key)
        if ctx is not None:
            return ctx
        if not torch.cuda.is_available():
            raise RuntimeError("gaussiansplattingviewer_amd needs a HIP device (MI355X); "
                               "torch.cuda.is_available() is False")
        if key[1] == 0 and _native_shares_library():
            from . import _native  # owns (creates and destroys) the slot-0 contexts
            ctx = ctypes.c_void_p(_native.context_handle(key[0]))
        else:
            with torch.cuda.device(device_index):
                ctx = ctypes.c_void_p()
                check(lib.gsr_create(ctypes.byref(ctx)), "gsr_create")
        _contexts[key] = ctx
        return ctx


def release_contexts() -> None:
    """Destroy every gsr_context (registered with atexit; a diagnostics build reports its
    counters from gsr_destroy); slot 0's belong to `_native`."""
    with _lock:
        lib = _lib
        if lib is None or not _contexts:
            return
        native = _native_shares_library() and any(slot == 0 for _, slot in _contexts)
        for (_, slot), ctx in _contexts.items():
            if slot != 0 or not native:
                lib.gsr_destroy(ctx)
        _contexts.clear()
        if native:
            from . import _native
            _native.release_contexts()


atexit.register(release_contexts)


def frame_graph_stats(device_index: int = 0, slot: int = 0) -> dict:
    """Frame-graph counters of a context slot (gsr_frame_graph_stats)."""
    lib = load_library()
    v = (ctypes.c_int64 * 4)()
    check(lib.gsr_frame_graph_stats(context(device_index, slot), v, 4), "gsr_frame_graph_stats")
    return {"graph_frames": v[0], "graphs_recorded": v[1], "overflows": v[2], "list_cap": v[3]}


def get_option(ctx, option: int) -> int:
    """The current value of a context option (gsr_get_option)."""
    v = ctypes.c_int64()
    check(load_library().gsr_get_option(ctx, option, ctypes.byref(v)), "gsr_get_option")
    return int(v.value)


def set_option(ctx, option: int, value: int) -> None:
    check(load_library().gsr_set_option(ctx, option, int(value)), "gsr_set_option")


def stage_names() -> list[str]:
    lib = load_library()
    names = []
    i = 0
    while True:
        n = lib.gsr_stage_name(i).decode()
        if not n:
            return names
        names.append(n)
        i += 1


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for an absent / empty optional tensor)."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()
