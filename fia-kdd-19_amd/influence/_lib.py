"""ctypes binding of libfia.so (include/fia.h) for torch device tensors.

This is the ONLY compute path of the package: there is no CPU fallback.  If
the library is missing (not built) or no GPU is visible, every entry point
raises, loudly.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FIA_LIB", os.path.join(_HERE, "libfia.so"))

FIA_OK = 0
FIA_MODEL_MF = 0
FIA_MODEL_NCF = 1
FIA_MAX_TOPK = 64
FIA_NUM_PHASES = 5
PHASES = ("prepare", "solve", "score", "topk", "chunks")

_ERR = {1: "invalid argument", 2: "HIP error", 3: "bad call order", 4: "unsupported", 5: "out of memory"}

# exported symbol -> (restype, argtypes); every symbol declared in include/fia.h
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
SIGNATURES = {
    "fia_version": (ctypes.c_int, []),
    "fia_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "fia_destroy": (ctypes.c_int, [_P]),
    "fia_last_error": (ctypes.c_char_p, [_P]),
    "fia_set_params": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _I64, _I64, ctypes.POINTER(_P), ctypes.c_int,
                                      ctypes.c_double, ctypes.c_double]),
    "fia_build_index": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _P, _P, _P]),
    "fia_prepare": (ctypes.c_int, [_P, _P]),
    "fia_prepare_for": (ctypes.c_int, [_P, _I64, _P, _P, _P]),
    "fia_count_related": (ctypes.c_int, [_P, _I64, _P, _P, _P, ctypes.POINTER(_I64), _P]),
    "fia_related": (ctypes.c_int, [_P, _I64, _P, _P, _P, _P, _P]),
    "fia_query_batch": (ctypes.c_int, [_P, _I64, _P, _P, _P, _I64, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P]),
    "fia_query_batch_x": (ctypes.c_int, [_P, _I64, _P, _P, _P, _I64, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P]),
    "fia_num_params": (ctypes.c_int, [_P]),
    "fia_set_profiling": (ctypes.c_int, [_P, ctypes.c_int]),
    "fia_profile_read": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64)]),
}

_lib = None


class FIAError(RuntimeError):
    pass


def load_library(path=None):
    """dlopen libfia.so and bind every symbol (no GPU needed for this step)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError("FIA HIP library not built: %s is missing (run __graft_entry__.build() or "
                          "make -C fia-kdd-19_amd/csrc)" % p)
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Context(object):
    """One fia_ctx bound to one HIP device."""

    def __init__(self, device=0):
        import torch
        if not torch.cuda.is_available():
            raise FIAError("FIA needs a ROCm GPU: torch.cuda.is_available() is False (no CPU fallback)")
        self.lib = load_library()
        self.device = device
        self.torch_device = torch.device("cuda", device)
        h = ctypes.c_void_p()
        rc = self.lib.fia_create(device, ctypes.byref(h))
        if rc != FIA_OK:
            raise FIAError("fia_create(%d) failed: %s" % (device, _ERR.get(rc, rc)))
        self.h = h
        self._keep = []
        self._mask = 0
        self._carry = None      # phase sums drained by profiled_call on the caller's behalf
        self.full_prepared = False   # every entity's caches (the last prepare was fia_prepare)

    def close(self):
        if getattr(self, "h", None):
            self.lib.fia_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != FIA_OK:
            msg = self.lib.fia_last_error(self.h)
            raise FIAError("%s failed (%s): %s" % (what, _ERR.get(rc, rc), msg.decode() if msg else ""))

    # ---- setup ----
    def set_params(self, model, k, U, I, tables, wd, damping):
        """tables: list of contiguous float32 cuda tensors in include/fia.h order."""
        arr = (ctypes.c_void_p * len(tables))(*[t.data_ptr() for t in tables])
        self._keep = list(tables)
        self.full_prepared = False
        self._num_params = None
        rc = self.lib.fia_set_params(self.h, model, k, U, I, arr, len(tables), float(wd), float(damping))
        self._check(rc, "fia_set_params")

    def build_index(self, users, items, ratings, U, I):
        self.full_prepared = False
        rc = self.lib.fia_build_index(self.h, users.numel(), U, I, _ptr(users), _ptr(items), _ptr(ratings),
                                      _stream())
        self._check(rc, "fia_build_index")

    def prepare(self):
        self.full_prepared = False
        self._check(self.lib.fia_prepare(self.h, _stream()), "fia_prepare")
        self.full_prepared = True

    def prepare_for(self, qu, qi):
        """Hessian caches for only the users/items of these queries (fia_prepare_for, every
        model: small k marks the entities on the device, large k builds a compact cache)."""
        self.full_prepared = False
        self._check(self.lib.fia_prepare_for(self.h, qu.numel(), _ptr(qu), _ptr(qi), _stream()), "fia_prepare_for")

    def num_params(self):
        if getattr(self, "_num_params", None) is None:
            self._num_params = self.lib.fia_num_params(self.h)
        return self._num_params

    # ---- queries ----
    def count_related(self, qu, qi, offsets=None, want_total=True):
        import torch
        Q = qu.numel()
        if offsets is None:
            offsets = torch.empty(Q + 1, dtype=torch.int64, device=self.torch_device)
        total = ctypes.c_int64(0)
        rc = self.lib.fia_count_related(self.h, Q, _ptr(qu), _ptr(qi), _ptr(offsets),
                                        ctypes.byref(total) if want_total else None, _stream())
        self._check(rc, "fia_count_related")
        return offsets, (total.value if want_total else None)

    @staticmethod
    def _need_int32(t, name):
        # the library writes train rows as int32 (include/fia.h fia_related)
        import torch
        if t is not None and t.dtype != torch.int32:
            raise TypeError("%s must be a torch.int32 tensor (got %s)" % (name, t.dtype))

    def related(self, qu, qi, offsets, rel_idx):
        self._need_int32(rel_idx, "rel_idx")
        rc = self.lib.fia_related(self.h, qu.numel(), _ptr(qu), _ptr(qi), _ptr(offsets), _ptr(rel_idx), _stream())
        self._check(rc, "fia_related")

    def query_batch(self, qu, qi, offsets, total, rel_idx=None, influence=None, x=None, K=0,
                    topk_pos=None, topk_idx=None, topk_val=None):
        self._need_int32(rel_idx, "rel_idx")
        rc = self.lib.fia_query_batch(self.h, qu.numel(), _ptr(qu), _ptr(qi), _ptr(offsets), int(total),
                                      _ptr(rel_idx), _ptr(influence), _ptr(x), int(K), _ptr(topk_pos),
                                      _ptr(topk_idx), _ptr(topk_val), _stream())
        self._check(rc, "fia_query_batch")

    def query_batch_x(self, qu, qi, offsets, total, x_in, rel_idx=None, influence=None, K=0,
                      topk_pos=None, topk_idx=None, topk_val=None):
        """fia_query_batch with the given inverse HVPs x_in (float64 cuda tensor [Q * D],
        reference theta order) instead of the solve."""
        import torch
        self._need_int32(rel_idx, "rel_idx")
        if x_in.dtype != torch.float64 or not x_in.is_contiguous():
            raise TypeError("x_in must be a contiguous torch.float64 tensor")
        if not x_in.is_cuda:
            raise TypeError("x_in must be a device (cuda) tensor")
        if x_in.numel() < qu.numel() * self.num_params():
            raise ValueError("x_in holds %d values, %d queries need %d" % (
                x_in.numel(), qu.numel(), qu.numel() * self.num_params()))
        rc = self.lib.fia_query_batch_x(self.h, qu.numel(), _ptr(qu), _ptr(qi), _ptr(offsets), int(total),
                                        _ptr(x_in), _ptr(rel_idx), _ptr(influence), int(K), _ptr(topk_pos),
                                        _ptr(topk_idx), _ptr(topk_val), _stream())
        self._check(rc, "fia_query_batch_x")

    # ---- profiling ----
    def set_profiling(self, on, phases=None):
        """on: record HIP-event pairs for the phases named in `phases` (all if None)."""
        mask = 0
        if on:
            mask = 0x1f if phases is None else sum(1 << PHASES.index(p) for p in phases)
        self._set_mask(mask)

    def _set_mask(self, mask):
        self._check(self.lib.fia_set_profiling(self.h, mask), "fia_set_profiling")
        self._mask = mask
        if mask:
            self._pending = True    # events may be recorded until the next drain

    def _drain(self):
        ms = (ctypes.c_double * FIA_NUM_PHASES)()
        cnt = (ctypes.c_int64 * FIA_NUM_PHASES)()
        self._check(self.lib.fia_profile_read(self.h, ms, cnt), "fia_profile_read")
        self._pending = self._mask != 0
        return {PHASES[p]: (ms[p], cnt[p]) for p in range(FIA_NUM_PHASES)}

    def profile_read(self):
        """Per-phase (ms sum, count) recorded since the last read (synchronises the events)."""
        out = self._drain()
        if self._carry is not None:
            out = {p: (out[p][0] + self._carry[p][0], out[p][1] + self._carry[p][1]) for p in PHASES}
            self._carry = None
        return out

    def profiled_call(self, fn):
        """Run fn() with every phase recorded and return (fn's result, its phase sums).  The
        caller's profiling mask and the sums it has accumulated but not yet read are kept
        (the RQ2 timers of a single query, GenericNeuralNet.get_influence_on_test_loss)."""
        # (nothing can be pending when profiling was off since the last drain: skip that read)
        before = self._drain() if getattr(self, "_pending", True) else {p: (0.0, 0) for p in PHASES}
        mask = self._mask
        self._set_mask(0x1f)
        try:
            res = fn()
        finally:
            self._set_mask(mask)
        mine = self._drain()
        if self._carry is not None:
            before = {p: (before[p][0] + self._carry[p][0], before[p][1] + self._carry[p][1]) for p in PHASES}
        self._carry = before
        return res, mine
