"""mipgpu -- Python host side of the MI355X-native VVC MIP search engine.

Thin ctypes binding of ``libmipgpu.so`` (C ABI in ``include/mipgpu.h``).  The product
path is the HIP library only: if it is missing this module raises at import of
:class:`MipEngine` -- there is no CPU fallback.

Mirrors the reference's operator surface (main.cpp + main_aux_functions.h):
  * filter names / KernelIdx of the reference whitelist (constants.h:25-34),
  * the per-frame cost table in the reference layout (constants.h:1558-1631),
  * the CSV cost log is written by the C++ CLI (``bin/mipgpu_cli``, main_aux_functions.h:735-798).
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import sys
import weakref

import numpy as np

from . import layout
from .layout import COSTS_PER_CTU, CUS_PER_CTU, SHAPES, UNAVAILABLE, num_ctus

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MIPGPU_LIB", os.path.join(PKG_DIR, "lib", "libmipgpu.so"))

# Reference whitelist order (constants.h:25-34); index == mip_filter_type.
FILTERS = (
    "filterFrame_1d_int",
    "filterFrame_1d_float",
    "filterFrame_2d_int_quarterCtu",
    "filterFrame_2d_float_quarterCtu",
    "filterFrame_1d_int_5x5",
    "filterFrame_1d_float_5x5",
    "filterFrame_2d_int_5x5_quarterCtu",
    "filterFrame_2d_float_5x5_quarterCtu",
)
FILTER_NONE = -1


class MipError(RuntimeError):
    pass


def filter_index(name) -> int:
    """Filter name (reference spelling) or index -> mip_filter_type; None -> FILTER_NONE."""
    if name is None:
        return FILTER_NONE
    if isinstance(name, (int, np.integer)):
        return int(name)
    if name not in FILTERS:
        raise MipError(f"Filter type {name} not supported")  # main.cpp:74-76
    return FILTERS.index(name)


class _Opts(ctypes.Structure):
    _fields_ = [("filter", ctypes.c_int), ("kernel_idx", ctypes.c_int), ("max_batch", ctypes.c_int),
                ("want_sad_satd", ctypes.c_int), ("slices_per_ctu", ctypes.c_int), ("best_k", ctypes.c_int)]


_lib = None


def _torch_hip_runtime():
    """Path of the HIP runtime bundled in torch's ROCm wheel (torch/lib/libamdhip64.so), or None
    when torch is not installed or bundles none -- found without importing torch."""
    spec = importlib.util.find_spec("torch")
    for d in (spec.submodule_search_locations or []) if spec is not None else []:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            return p
    return None


def _one_hip_runtime():
    """One HIP runtime per process.  torch's ROCm wheel bundles its own libamdhip64 /
    libhsa-runtime64 and loads them by path, so if libmipgpu.so bound /opt/rocm's runtime a
    later `import torch` would bring a second HIP and HSA runtime into the process, and torch
    then finds no GPU once ours has opened it.  So when torch is installed, its bundled
    runtime is loaded first -- by path, with RTLD_GLOBAL, without importing torch (a
    multi-second import with process-wide side effects that numpy-only callers and the CLI
    wrappers do not need) -- and libmipgpu.so binds to it (same soname, libamdhip64.so.7); a
    later `import torch` finds it already mapped.  MIPGPU_NO_TORCH=1 skips this (a process
    that never imports torch: /opt/rocm's runtime)."""
    if "torch" in sys.modules or os.environ.get("MIPGPU_NO_TORCH"):
        return
    path = _torch_hip_runtime()
    if path is not None:
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def hip_runtimes():
    """Paths of the HIP runtime libraries mapped into this process (diagnostic: one expected)."""
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})


def library():
    """Load libmipgpu.so (raises if it was not built: the HIP path is mandatory)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MipError(f"{LIB_PATH} not found -- build it with `make -C vvc-mip-gpu_amd` "
                       "(or __graft_entry__.build()); there is no CPU fallback")
    _one_hip_runtime()
    L = ctypes.CDLL(LIB_PATH)
    vp, ip, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    sig = {
        "mip_opts_default": (None, [ctypes.POINTER(_Opts)]),
        "mip_engine_create": (ip, [ip, ip, ip, ctypes.POINTER(_Opts), ctypes.POINTER(vp)]),
        "mip_engine_destroy": (ip, [vp]),
        "mip_num_ctus": (ip, [ip, ip]),
        "mip_costs_per_frame": (i64, [ip, ip]),
        "mip_cus_per_frame": (i64, [ip, ip]),
        "mip_shape_name": (ctypes.c_char_p, [ip]),
        "mip_shape_info": (ip, [ip] + [ctypes.POINTER(ip)] * 5),
        "mip_cu_position": (ip, [ip, ip, ctypes.POINTER(ip), ctypes.POINTER(ip)]),
        "mip_filter_frames": (ip, [vp, vp, ip, ip, ip, vp]),
        "mip_search_frames": (ip, [vp, vp, vp, ip, vp, vp, vp, vp, vp]),
        "mip_search_frames_async": (ip, [vp, vp, vp, ip, vp, vp, vp, vp, vp, ctypes.POINTER(ctypes.c_uint64)]),
        "mip_wait": (ip, [vp, ctypes.c_uint64]),
        "mip_flush": (ip, [vp]),
        "mip_device_cache": (ip, [ip, ip, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "mip_search_device": (ip, [vp, vp, vp, ip, vp, vp, vp, vp, vp, vp]),
        "mip_search_device_range": (ip, [vp, vp, vp, ip, ip, ip, vp, vp, vp, vp]),
        "mip_check_input": (ip, [vp, vp]),
        "mip_unavailable_cus": (ip, [ip, ip, ip, vp]),
        "mip_filter_device": (ip, [vp, vp, ip, ip, ip, ip, ip, vp]),
        "mip_copy_device": (ip, [vp, vp, ctypes.c_size_t, vp]),
        "mip_topk_device": (ip, [vp, ip, ip, ip, ip, vp, vp, vp]),
        "mip_time_search_device": (ctypes.c_double, [vp, vp, vp, ip, vp, ip]),
        "mip_host_stats": (ip, [vp, ctypes.POINTER(ctypes.c_uint64), ip]),
        "mip_host_alloc": (ip, [ctypes.c_size_t, ctypes.POINTER(vp)]),
        "mip_host_free": (ip, [vp]),
        "mip_host_alloc_near": (ip, [ip, ctypes.c_size_t, ctypes.POINTER(vp)]),
        "mip_bind_thread": (ip, [ip]),
        "mip_numa_node": (ip, [ip]),
        "mip_numa_node_of_pci": (ip, [ctypes.c_char_p]),
        "mip_last_error": (ctypes.c_char_p, []),
        "mip_abi_version": (ip, []),
        "mip_build_id": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def build_id() -> str:
    """mip_build_id(): 'src:<source + flag hash> git:<commit>[ knobs:...]'."""
    return library().mip_build_id().decode()


def source_id(bid: str) -> str:
    """The part of a build ID that identifies the compiled code (the 'src:' token)."""
    return bid.split()[0] if bid else ""


def _check(rc):
    if rc != 0:
        raise MipError(library().mip_last_error().decode())


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


def pinned_empty(shape, dtype, device=None) -> np.ndarray:
    """Uninitialised numpy array in page-locked host memory (mip_host_alloc; with `device`,
    mip_host_alloc_near: on that GPU's NUMA node); transfers to / from it run at DMA rate.
    The memory is released with the last view of it."""
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    p = ctypes.c_void_p()
    if device is None:
        _check(library().mip_host_alloc(max(1, count * dt.itemsize), ctypes.byref(p)))
    else:
        _check(library().mip_host_alloc_near(int(device), max(1, count * dt.itemsize), ctypes.byref(p)))
    buf = (ctypes.c_byte * max(1, count * dt.itemsize)).from_address(p.value)
    weakref.finalize(buf, library().mip_host_free, ctypes.c_void_p(p.value))
    return np.frombuffer(buf, dtype=dt, count=count).reshape(shape)


class _Ticket:
    """An asynchronous host search in flight: its number, its outputs, and its inputs (kept
    alive until the search has completed).  A ticket dropped without wait() waits in its
    finaliser, so numpy never frees arrays the engine's copies may still be using.  The
    finaliser may run on any thread (garbage collection): it takes the engine's lock, like
    every engine call, because mip_wait drains the engine's bounce ring (not thread safe)."""

    def __init__(self, value, out, keep, engine=None):
        self.value, self.out, self._keep, self._engine = value, out, keep, engine
        self.done = engine is None

    def __del__(self):
        eng = getattr(self, "_engine", None)
        if getattr(self, "done", True) or eng is None:
            return
        try:
            with eng._lock:
                if getattr(eng, "_h", None) and library().mip_wait(eng._h, ctypes.c_uint64(self.value)) != 0:
                    # a finaliser cannot raise: a dropped call's error (e.g. the input contract,
                    # reported per call by mip_wait) becomes a warning instead of vanishing
                    import warnings
                    warnings.warn("dropped search ticket %d failed: %s" % (self.value, library().mip_last_error().decode()),
                                  RuntimeWarning, stacklevel=2)
        except Exception:
            pass


class MipEngine:
    """One engine per GPU (mip_engine_create).  Calls on one engine are serialised by a
    per-engine lock (the C engine must be used by one thread at a time); use one engine per
    thread for concurrency."""

    def __init__(self, width: int, height: int, device: int = 0, filter=None, kernel_idx: int = 0,
                 max_batch: int = 1, want_sad_satd: bool = False, slices_per_ctu: int = 0, best_k: int = 1):
        import threading
        self._lock = threading.RLock()
        L = library()
        self.width, self.height = int(width), int(height)
        self.nctus = num_ctus(self.width, self.height)
        self.filter = filter_index(filter)
        self.kernel_idx = int(kernel_idx)
        self.max_batch = int(max_batch)
        self.want_sad_satd = bool(want_sad_satd)
        self.best_k = int(best_k)
        o = _Opts(self.filter, self.kernel_idx, self.max_batch, int(self.want_sad_satd), int(slices_per_ctu),
                  self.best_k)
        h = ctypes.c_void_p()
        _check(L.mip_engine_create(int(device), self.width, self.height, ctypes.byref(o), ctypes.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        lock = getattr(self, "_lock", None)
        if lock is None:
            return
        with lock:
            if getattr(self, "_h", None):
                library().mip_engine_destroy(self._h)  # synchronises the engine streams first
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def costs_per_frame(self) -> int:
        return self.nctus * COSTS_PER_CTU

    @property
    def cus_per_frame(self) -> int:
        return self.nctus * CUS_PER_CTU

    # ---------------------------------------------------------------- host API
    def _frames(self, frames):
        f = np.ascontiguousarray(frames, dtype=np.uint16)
        if f.ndim == 2:
            f = f[None]
        if f.shape[1:] != (self.height, self.width):
            raise MipError(f"frames of shape {f.shape[1:]} do not match {self.height}x{self.width}")
        return f

    def search(self, frames, refs=None, costs=True, best=False, sad_satd=False, out=None):
        """Full MIP search of host frames ([F,H,W] or [H,W] uint16).  Returns a dict with
        'cost' [F, nCTUs*97840] int32 and optionally 'best_mode' / 'best_cost' [F, nCTUs*5380]
        (decision lists [F, nCTUs*5380, K] when the engine has best_k = K > 1), 'sad' / 'satd'.
        `out` may supply any of these arrays (e.g. from pinned_empty, for DMA-rate
        transfers); the others are allocated."""
        f, r, n, res = self._prepare(frames, refs, costs, best, sad_satd, out)
        with self._lock:  # mip_search_frames: one synchronous call (its last chunks may ramp down)
            _check(library().mip_search_frames(self._h, _ptr(f), _ptr(r), n, _ptr(res.get("cost")),
                                               _ptr(res.get("best_mode")), _ptr(res.get("best_cost")),
                                               _ptr(res.get("sad")), _ptr(res.get("satd"))))
        return res

    def search_async(self, frames, refs=None, costs=True, best=False, sad_satd=False, out=None):
        """As search(), without waiting (mip_search_frames_async): the call queues behind
        the calls in flight and returns a ticket; wait(ticket) returns the output dict.  The
        ticket keeps the input and output arrays alive until then."""
        f, r, n, res = self._prepare(frames, refs, costs, best, sad_satd, out)
        t = ctypes.c_uint64()
        with self._lock:
            _check(library().mip_search_frames_async(self._h, _ptr(f), _ptr(r), n, _ptr(res.get("cost")),
                                                     _ptr(res.get("best_mode")), _ptr(res.get("best_cost")),
                                                     _ptr(res.get("sad")), _ptr(res.get("satd")), ctypes.byref(t)))
        return _Ticket(t.value, res, (f, r), self)

    def _prepare(self, frames, refs, costs, best, sad_satd, out):
        """Input arrays and the output dict of a host search (allocated unless in `out`)."""
        f = self._frames(frames)
        r = None if refs is None else self._frames(refs)
        n = f.shape[0]
        given = dict(out or {})

        def buf(key, want, cols, dtype):
            if not want:
                return None
            shape = (n,) + (cols if isinstance(cols, tuple) else (cols,))
            a = given.get(key)
            if a is None:
                return np.empty(shape, dtype)
            if a.dtype != np.dtype(dtype) or a.shape != shape or not a.flags.c_contiguous:
                raise MipError(f"out[{key!r}] must be a C-contiguous {np.dtype(dtype)} array of shape {shape}")
            return a

        res = {}
        bcols = self.cus_per_frame if self.best_k == 1 else (self.cus_per_frame, self.best_k)
        for key, want, cols, dt in (("cost", costs, self.costs_per_frame, np.int32),
                                    ("best_mode", best, bcols, np.uint8), ("best_cost", best, bcols, np.int32),
                                    ("sad", sad_satd, self.costs_per_frame, np.int32),
                                    ("satd", sad_satd, self.costs_per_frame, np.int32)):
            a = buf(key, want, cols, dt)
            if a is not None:
                res[key] = a
        return f, r, n, res

    def wait(self, ticket):
        """Block until an asynchronous search has completed; returns its output dict."""
        with self._lock:
            ticket.done = True  # also on error: the call is over either way
            _check(library().mip_wait(self._h, ctypes.c_uint64(ticket.value)))
        return ticket.out

    def host_stats(self) -> dict:
        """Host-pipeline counters (mip_host_stats): calls, search launches, calls that went
        through merged launches, merged launches."""
        out = (ctypes.c_uint64 * 4)()
        with self._lock:
            _check(library().mip_host_stats(self._h, out, 4))
        return dict(zip(("calls", "launches", "merged_calls", "merged_launches"), (int(v) for v in out)))

    def flush(self):
        """Launch the engine's open (merged) chunk now (mip_flush): queued small calls are
        otherwise launched by the next call, a wait, or when the chunk is full."""
        with self._lock:
            _check(library().mip_flush(self._h))

    def filter_frames(self, frames, filter, kernel_idx=0):
        f = self._frames(frames)
        out = np.empty_like(f)
        with self._lock:
            _check(library().mip_filter_frames(self._h, _ptr(f), f.shape[0], filter_index(filter), int(kernel_idx),
                                               _ptr(out)))
        return out

    # -------------------------------------------------------------- device API
    def search_device(self, frames, refs=None, costs=None, sad=None, satd=None, best_mode=None,
                      best_cost=None, stream=None):
        """Asynchronous search on device tensors (torch, int16/uint16 [F,H,W]) on `stream`
        (a torch.cuda.Stream; default: torch's current stream).  costs=False: decisions only
        (no cost table; needs best_cost, best_k = 1; returns None)."""
        import torch
        n = frames.shape[0]
        if costs is False:
            costs = None
        elif costs is None:
            costs = torch.empty((n, self.costs_per_frame), dtype=torch.int32, device=frames.device)
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        with self._lock:
            _check(library().mip_search_device(self._h, _ptr(frames), _ptr(refs), n, _ptr(costs), _ptr(sad),
                                               _ptr(satd), _ptr(best_mode), _ptr(best_cost),
                                               ctypes.c_void_p(s.cuda_stream)))
        return costs

    def search_device_range(self, frames, ctu_begin, ctu_end, costs, refs=None, sad=None, satd=None, stream=None):
        """search_device over the CTUs [ctu_begin, ctu_end) of every frame only
        (mip_search_device_range): their blocks of the full-size `costs` are written."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        with self._lock:
            _check(library().mip_search_device_range(self._h, _ptr(frames), _ptr(refs), frames.shape[0],
                                                     int(ctu_begin), int(ctu_end), _ptr(costs), _ptr(sad), _ptr(satd),
                                                     ctypes.c_void_p(s.cuda_stream)))
        return costs

    def check_input(self, stream=None):
        """Input contract of the device-API searches on `stream` (mip_check_input): waits for
        the stream and raises MipError if a search staged a sample above 1023 (10 bits)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        with self._lock:
            _check(library().mip_check_input(self._h, ctypes.c_void_p(s.cuda_stream)))

    def time_search_device(self, frames, costs, refs=None, reps=10) -> float:
        with self._lock:
            ms = library().mip_time_search_device(self._h, _ptr(frames), _ptr(refs), frames.shape[0], _ptr(costs),
                                                  int(reps))
        if ms < 0:
            raise MipError(library().mip_last_error().decode())
        return ms


def device_cache(device=0, release=False) -> dict:
    """The process-wide device block cache (mip_device_cache): bytes parked for `device` by
    destroyed engines and blocks reused so far; release=True frees the parked blocks first."""
    idle, reused = ctypes.c_uint64(), ctypes.c_uint64()
    _check(library().mip_device_cache(int(device), int(bool(release)), ctypes.byref(idle), ctypes.byref(reused)))
    return {"idle_bytes": int(idle.value), "reused_blocks": int(reused.value)}


def numa_node(device) -> int:
    """NUMA node of a GPU (mip_numa_node; -1: unknown or a one-node host)."""
    return int(library().mip_numa_node(int(device)))


def bind_thread(device) -> bool:
    """Run the calling thread on the CPUs of the GPU's NUMA node (mip_bind_thread)."""
    return library().mip_bind_thread(int(device)) == 1


def unavailable_cus(width, height, filter=None) -> np.ndarray:
    """Bool per CU (reference order): the CUs an engine with this filter reports as
    MIP_COST_UNAVAILABLE (mip_unavailable_cus; host only)."""
    n = num_ctus(width, height) * CUS_PER_CTU
    out = np.zeros(n, np.uint8)
    _check(library().mip_unavailable_cus(int(width), int(height), filter_index(filter), out.ctypes.data))
    return out.astype(bool)


def topk_device(costs, width, height, k, modes=None, costs_k=None, stream=None):
    """Per-CU decision lists of device cost tables (torch int32 [F, nCTUs*97840]):
    returns (modes uint8, costs int32), each [F, nCTUs*5380, k] (mip_topk_device)."""
    import torch
    n = costs.shape[0]
    shape = (n, num_ctus(width, height) * CUS_PER_CTU, int(k))
    if modes is None:
        modes = torch.empty(shape, dtype=torch.uint8, device=costs.device)
    if costs_k is None:
        costs_k = torch.empty(shape, dtype=torch.int32, device=costs.device)
    s = stream if stream is not None else torch.cuda.current_stream(costs.device)
    _check(library().mip_topk_device(_ptr(costs), int(width), int(height), n, int(k), _ptr(modes), _ptr(costs_k),
                                     ctypes.c_void_p(s.cuda_stream)))
    return modes, costs_k


def copy_device(src, dst, stream=None):
    """Streaming device copy of tensor `src` into `dst` (mip_copy_device; same byte size)."""
    import torch
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != n:
        raise MipError("copy_device: sizes differ")
    s = stream if stream is not None else torch.cuda.current_stream(src.device)
    _check(library().mip_copy_device(_ptr(src), _ptr(dst), n, ctypes.c_void_p(s.cuda_stream)))
    return dst


def filter_device(frames_in, frames_out, filter, kernel_idx=0, stream=None):
    import torch
    n, h, w = frames_in.shape
    s = stream if stream is not None else torch.cuda.current_stream(frames_in.device)
    _check(library().mip_filter_device(_ptr(frames_in), _ptr(frames_out), w, h, n, filter_index(filter),
                                       int(kernel_idx), ctypes.c_void_p(s.cuda_stream)))
    return frames_out


__all__ = ["MipEngine", "MipError", "build_id", "source_id", "FILTERS", "FILTER_NONE", "filter_index", "filter_device", "topk_device", "library",
           "pinned_empty", "unavailable_cus", "numa_node", "bind_thread", "device_cache", "copy_device",
           "layout", "SHAPES", "COSTS_PER_CTU", "CUS_PER_CTU", "UNAVAILABLE", "num_ctus"]
