"""ctypes binding of libemrifd.so (the C ABI declared in include/emrifd.h).

This is the only way the package reaches its compute path. There is deliberately no CPU
fallback: if the HIP library is missing or no GPU is visible, calls raise.
"""

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EFD_LIB") or os.path.join(_HERE, "libemrifd.so")

EFD_OK = 0
EFD_ERR_ARG = -1
EFD_ERR_HIP = -2
EFD_ERR_WORKSPACE = -3
EFD_CAUSTIC_SPA = 0
EFD_CAUSTIC_UNIFORM = 1
EFD_LOGLIKE_SCRATCH = 1024
EFD_INNER_SCRATCH = 2048
EFD_BATCH_MAX = 16
EFD_HANN_ROWS_MAX = 16   # efd_hann_loglike's rows per call (include/emrifd.h)
EFD_HANN_LOCAL_PARTIALS = 4096   # efd_hann_loglike_local's scratch doubles per row

# every symbol include/emrifd.h declares (tests check the library exports all of them)
EXPORTED_SYMBOLS = (
    "efd_version",
    "efd_build_id",
    "efd_last_error",
    "efd_spline_build",
    "efd_modesum_workspace_bytes",
    "efd_modesum",
    "efd_modesum_prepare",
    "efd_modesum_prepare_batch",
    "efd_modesum_status_batch",
    "efd_stage_batch",
    "efd_fused_group",
    "efd_modesum_sum",
    "efd_modesum_sum_batch",
    "efd_modesum_sum_loglike",
    "efd_loglike_tile_count",
    "efd_loglike_tile_constants",
    "efd_modesum_sum_loglike_ex",
    "efd_modesum_status",
    "efd_modesum_contributions",
    "efd_modesum_stats",
    "efd_modesum_env_evaluations",
    "efd_td_workspace_bytes",
    "efd_td_modesum",
    "efd_upload",
    "efd_download",
    "efd_stream_order",
    "efd_polarizations",
    "efd_modesum_lane_ranges",
    "efd_hann_extent",
    "efd_hann_stage",
    "efd_hann_convolve",
    "efd_hann_four_step_cols",
    "efd_hann_polarizations",
    "efd_hann_loglike",
    "efd_hann_loglike_local",
    "efd_hann_loglike_local_partials",
    "efd_loglike",
    "efd_inner_product",
    "efd_modesum_cpu",
    "efd_modesum_cpu_stats",
    "efd_spline_build_cpu",
    "efd_polarizations_cpu",
    "efd_loglike_cpu",
    "efd_inner_product_cpu",
    "efd_cpu_threads",
    "efd_cpu_last_error",
    "efd_host_trajectory",
    "efd_host_p_at_t",
    "efd_host_modes",
    "efd_host_set_threads",
)


class ModesumArgs(ctypes.Structure):
    """Mirror of `efd_modesum_args` (include/emrifd.h)."""

    _fields_ = [
        ("t", ctypes.c_void_p),
        ("phi_phi", ctypes.c_void_p),
        ("phi_r", ctypes.c_void_p),
        ("f_phi", ctypes.c_void_p),
        ("f_r", ctypes.c_void_p),
        ("nt", ctypes.c_int32),
        ("amp", ctypes.c_void_p),
        ("m", ctypes.c_void_p),
        ("n", ctypes.c_void_p),
        ("ylm_p", ctypes.c_void_p),
        ("ylm_m", ctypes.c_void_p),
        ("K", ctypes.c_int32),
        ("freq", ctypes.c_void_p),
        ("nf", ctypes.c_int64),
        ("grid_symmetric", ctypes.c_int32),
        ("scale_re", ctypes.c_double),
        ("scale_im", ctypes.c_double),
        ("caustic", ctypes.c_int32),
        ("accumulate", ctypes.c_int32),
        ("out", ctypes.c_void_p),
        ("prof_begin", ctypes.c_void_p),
        ("prof_end", ctypes.c_void_p),
        ("hp", ctypes.c_void_p),
        ("hc", ctypes.c_void_p),
        ("k0", ctypes.c_int64),
    ]


class TdArgs(ctypes.Structure):
    """Mirror of `efd_td_args` (include/emrifd.h)."""

    _fields_ = [
        ("t", ctypes.c_void_p),
        ("phi_phi", ctypes.c_void_p),
        ("phi_r", ctypes.c_void_p),
        ("f_phi", ctypes.c_void_p),
        ("f_r", ctypes.c_void_p),
        ("nt", ctypes.c_int32),
        ("amp", ctypes.c_void_p),
        ("m", ctypes.c_void_p),
        ("n", ctypes.c_void_p),
        ("ylm_p", ctypes.c_void_p),
        ("ylm_m", ctypes.c_void_p),
        ("K", ctypes.c_int32),
        ("dt", ctypes.c_double),
        ("nsamples", ctypes.c_int64),
        ("scale_re", ctypes.c_double),
        ("scale_im", ctypes.c_double),
        ("accumulate", ctypes.c_int32),
        ("out", ctypes.c_void_p),
        ("hp", ctypes.c_void_p),
        ("hc", ctypes.c_void_p),
        ("prof_begin", ctypes.c_void_p),
        ("prof_end", ctypes.c_void_p),
    ]


class EFDError(RuntimeError):
    pass


_lib = None


def load(path=None):
    """Load libemrifd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    try:  # load torch's HIP runtime first so libemrifd.so binds to the same libamdhip64.so.7
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise EFDError(
            f"HIP library {p} not found: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(p)
    vp, i32, i64, dbl, sz = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double,
                             ctypes.c_size_t)
    lib.efd_version.restype = ctypes.c_int
    lib.efd_version.argtypes = []
    lib.efd_build_id.restype = ctypes.c_char_p
    lib.efd_build_id.argtypes = []
    lib.efd_last_error.restype = ctypes.c_int
    lib.efd_last_error.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.efd_spline_build.restype = ctypes.c_int
    lib.efd_spline_build.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, vp]
    lib.efd_modesum_workspace_bytes.restype = sz
    lib.efd_modesum_workspace_bytes.argtypes = [i32, i32, i64]
    lib.efd_modesum.restype = ctypes.c_int
    lib.efd_modesum.argtypes = [ctypes.POINTER(ModesumArgs), vp, sz, vp]
    for name in ("efd_modesum_prepare", "efd_modesum_sum"):
        if hasattr(lib, name):   # absent only in older experiment builds
            getattr(lib, name).restype = ctypes.c_int
            getattr(lib, name).argtypes = [ctypes.POINTER(ModesumArgs), vp, sz, vp]
    if hasattr(lib, "efd_modesum_prepare_batch"):
        lib.efd_modesum_prepare_batch.restype = ctypes.c_int
        lib.efd_modesum_prepare_batch.argtypes = [ctypes.POINTER(ctypes.POINTER(ModesumArgs)),
                                                  ctypes.POINTER(vp), ctypes.POINTER(sz), i32, vp]
    if hasattr(lib, "efd_modesum_sum_batch"):
        lib.efd_modesum_sum_batch.restype = ctypes.c_int
        lib.efd_modesum_sum_batch.argtypes = [ctypes.POINTER(ctypes.POINTER(ModesumArgs)),
                                              ctypes.POINTER(vp), ctypes.POINTER(sz), i32, vp]
    if hasattr(lib, "efd_modesum_sum_loglike"):
        lib.efd_modesum_sum_loglike.restype = ctypes.c_int
        lib.efd_modesum_sum_loglike.argtypes = [ctypes.POINTER(ctypes.POINTER(ModesumArgs)),
                                                ctypes.POINTER(vp), ctypes.POINTER(sz), i32, vp,
                                                vp, vp, vp]
    if hasattr(lib, "efd_modesum_sum_loglike_ex"):
        lib.efd_loglike_tile_count.restype = i64
        lib.efd_loglike_tile_count.argtypes = [i64]
        lib.efd_loglike_tile_constants.restype = ctypes.c_int
        lib.efd_loglike_tile_constants.argtypes = [vp, vp, i64, i64, vp, vp]
        lib.efd_modesum_sum_loglike_ex.restype = ctypes.c_int
        lib.efd_modesum_sum_loglike_ex.argtypes = [ctypes.POINTER(ctypes.POINTER(ModesumArgs)),
                                                   ctypes.POINTER(vp), ctypes.POINTER(sz), i32,
                                                   vp, vp, vp, vp, vp]
    lib.efd_modesum_status.restype = ctypes.c_int
    lib.efd_modesum_status.argtypes = [vp, vp]
    if hasattr(lib, "efd_stage_batch"):
        lib.efd_stage_batch.restype = ctypes.c_int
        lib.efd_stage_batch.argtypes = [vp, sz, ctypes.c_uint64, i32, vp, vp, vp,
                                        ctypes.POINTER(ModesumArgs), vp, ctypes.POINTER(sz)]
    if hasattr(lib, "efd_fused_group"):
        lib.efd_fused_group.restype = ctypes.c_int
        lib.efd_fused_group.argtypes = [vp, sz, vp, sz, i32, vp, vp, vp,
                                        ctypes.POINTER(ModesumArgs), vp, vp, vp, vp, vp, vp, vp,
                                        vp, vp, ctypes.POINTER(sz)]
    if hasattr(lib, "efd_modesum_status_batch"):
        lib.efd_modesum_status_batch.restype = ctypes.c_int
        lib.efd_modesum_status_batch.argtypes = [ctypes.POINTER(vp), i32, ctypes.POINTER(i32), vp]
    lib.efd_modesum_contributions.restype = ctypes.c_int
    lib.efd_modesum_contributions.argtypes = [vp, ctypes.POINTER(i64), vp]
    if hasattr(lib, "efd_modesum_stats"):   # absent only in pre-grouping experiment builds
        lib.efd_modesum_stats.restype = ctypes.c_int
        lib.efd_modesum_stats.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i64),
                                          ctypes.POINTER(i32), vp]
    if hasattr(lib, "efd_modesum_env_evaluations"):
        lib.efd_modesum_env_evaluations.restype = ctypes.c_int
        lib.efd_modesum_env_evaluations.argtypes = [vp, ctypes.POINTER(i64), vp]
    if hasattr(lib, "efd_td_modesum"):   # absent only in older experiment builds
        lib.efd_td_workspace_bytes.restype = sz
        lib.efd_td_workspace_bytes.argtypes = [i32, i32]
        lib.efd_td_modesum.restype = ctypes.c_int
        lib.efd_td_modesum.argtypes = [ctypes.POINTER(TdArgs), vp, sz, vp]
    if hasattr(lib, "efd_upload"):   # absent only in older experiment builds
        lib.efd_upload.restype = ctypes.c_int
        lib.efd_upload.argtypes = [vp, vp, sz, vp]
    if hasattr(lib, "efd_stream_order"):
        lib.efd_download.restype = ctypes.c_int
        lib.efd_download.argtypes = [vp, vp, sz, vp]
        lib.efd_stream_order.restype = ctypes.c_int
        lib.efd_stream_order.argtypes = [vp, ctypes.POINTER(vp), i32]
    lib.efd_polarizations.restype = ctypes.c_int
    lib.efd_polarizations.argtypes = [vp, i64, i64, vp, vp, vp]
    lib.efd_modesum_lane_ranges.restype = ctypes.c_int
    lib.efd_modesum_lane_ranges.argtypes = [vp, i32, vp, vp]
    lib.efd_hann_extent.restype = ctypes.c_int
    lib.efd_hann_extent.argtypes = [vp, i64, i64, i32, vp, vp, vp]
    lib.efd_hann_stage.restype = ctypes.c_int
    lib.efd_hann_stage.argtypes = [vp, i64, i64, i32, vp, i64, vp, vp]
    lib.efd_hann_convolve.restype = ctypes.c_int
    lib.efd_hann_convolve.argtypes = [vp, i64, i64, i32, vp, i64, vp, vp, vp]
    lib.efd_hann_four_step_cols.restype = ctypes.c_int
    lib.efd_hann_four_step_cols.argtypes = [i64]
    lib.efd_hann_polarizations.restype = ctypes.c_int
    lib.efd_hann_polarizations.argtypes = [vp, vp, vp, i64, i64, i64, vp, vp, vp]
    lib.efd_hann_loglike.restype = ctypes.c_int
    lib.efd_hann_loglike.argtypes = [vp, i64, vp, vp, i64, i32, i64, i64, vp, vp, vp, vp, vp]
    lib.efd_hann_loglike_local.restype = ctypes.c_int
    lib.efd_hann_loglike_local.argtypes = [vp, i64, i64, i32, vp, i64, vp, vp, vp, vp, i64, vp,
                                           vp, vp, vp]
    lib.efd_hann_loglike_local_partials.restype = ctypes.c_int
    lib.efd_hann_loglike_local_partials.argtypes = [i64]
    lib.efd_loglike.restype = ctypes.c_int
    lib.efd_loglike.argtypes = [vp, vp, vp, i32, i64, vp, vp, vp]
    lib.efd_inner_product.restype = ctypes.c_int
    lib.efd_inner_product.argtypes = [vp, vp, vp, i32, i64, vp, vp, vp]
    if hasattr(lib, "efd_modesum_cpu"):   # the host twins (csrc/emrifd_cpu.cpp)
        lib.efd_modesum_cpu.restype = ctypes.c_int
        lib.efd_modesum_cpu.argtypes = [ctypes.POINTER(ModesumArgs), vp, sz, vp]
        lib.efd_modesum_cpu_stats.restype = ctypes.c_int
        lib.efd_modesum_cpu_stats.argtypes = [ctypes.POINTER(i64), ctypes.POINTER(i64),
                                              ctypes.POINTER(i32)]
        lib.efd_spline_build_cpu.restype = ctypes.c_int
        lib.efd_spline_build_cpu.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, vp]
        lib.efd_polarizations_cpu.restype = ctypes.c_int
        lib.efd_polarizations_cpu.argtypes = [vp, i64, i64, vp, vp, vp]
        lib.efd_loglike_cpu.restype = ctypes.c_int
        lib.efd_loglike_cpu.argtypes = [vp, vp, vp, i32, i64, vp, vp, vp]
        lib.efd_inner_product_cpu.restype = ctypes.c_int
        lib.efd_inner_product_cpu.argtypes = [vp, vp, vp, i32, i64, vp, vp, vp]
        lib.efd_cpu_threads.restype = ctypes.c_int
        lib.efd_cpu_threads.argtypes = [ctypes.c_int]
        lib.efd_cpu_last_error.restype = ctypes.c_int
        lib.efd_cpu_last_error.argtypes = [ctypes.c_char_p, ctypes.c_int]
    if hasattr(lib, "efd_host_trajectory"):   # host upstream stand-ins (csrc/emrifd_host.cpp)
        lib.efd_host_trajectory.restype = ctypes.c_int
        lib.efd_host_trajectory.argtypes = [dbl] * 9 + [i32] + [vp] * 7 + [ctypes.POINTER(i32)]
        lib.efd_host_p_at_t.restype = ctypes.c_int
        lib.efd_host_p_at_t.argtypes = [dbl] * 10 + [ctypes.POINTER(dbl)]
        lib.efd_host_modes.restype = ctypes.c_int
        lib.efd_host_modes.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, i32, vp, vp, dbl, vp,
                                       ctypes.POINTER(i32), vp, i64]
        lib.efd_host_set_threads.restype = ctypes.c_int
        lib.efd_host_set_threads.argtypes = [i32]
        # the loading (main) thread's one-at-a-time upstream calls spread their knots over this
        # rank's host cores (hostcpu: its disjoint share of the node, not OMP_NUM_THREADS). The
        # setting is per thread: the prefetch pool's threads set their own per batch
        # (waveform.FastSchwarzschildEccentricFlux.prefetch splits the pool's threads over the
        # batch's walkers)
        import threading
        if threading.current_thread() is threading.main_thread():
            from . import hostcpu
            global _host_threads
            _host_threads = hostcpu.threads()
            lib.efd_host_set_threads(_host_threads)
    _ = dbl
    if path is None:
        _lib = lib
    return lib


_host_threads = 1


def host_threads():
    """The main thread's efd_host_set_threads value chosen by load() (hostcpu.threads())."""
    load()
    return _host_threads


def last_error(lib=None):
    lib = lib or load()
    buf = ctypes.create_string_buffer(512)
    lib.efd_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc, what, lib=None):
    if rc != EFD_OK:
        raise EFDError(f"{what} failed ({rc}): {last_error(lib)}")
    return rc
