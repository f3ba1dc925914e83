"""ctypes binding of libmoegan_hip.so (include/moegan_hip.h).

The HIP library is the product: there is no CPU or PyTorch fallback behind
these calls.  If the shared object is missing or fails to load, ``lib()``
raises -- the hot path fails loudly instead of silently running elsewhere.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MOEGAN_HIP_LIB") or os.path.join(_HERE, "libmoegan_hip.so")  # override: A/B builds

MG_F32, MG_BF16 = 0, 1
PREP_PACK, PREP_PACK_FLIP, PREP_PACK_DGRAD_S2, PREP_WSQ, PREP_WSQ_BWD, PREP_REPARAM = 1, 2, 3, 4, 5, 6
ACT_NONE, ACT_LRELU, ACT_GELU, ACT_MUL_GELU_GRAD, ACT_MUL_LRELU_GRAD, ACT_RSQRT_EPS, ACT_QUICK_GELU = range(7)

_c_void_p, _i32, _i64, _f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float


class Epilogue(ctypes.Structure):
    """Mirror of ``mg_epilogue`` (include/moegan_hip.h)."""
    _fields_ = [("alpha", _f32), ("bias", _c_void_p), ("scale", _c_void_p), ("scale_shift", _i32),
                ("scale_ld", _i64), ("rowscale", _c_void_p), ("act", _i32), ("aux", _c_void_p),
                ("ld_aux", _i64), ("resid", _c_void_p), ("ld_res", _i64), ("accumulate", _i32),
                ("atomic", _i32), ("remap_lgcin", _i32), ("remap_taps", _i32), ("a_idx", _c_void_p),
                ("a_idx_div", _i32), ("a_rowscale", _c_void_p), ("a_gelu", _i32), ("addvec", _c_void_p),
                ("add_shift", _i32), ("add_ld", _i64), ("out_pre", _c_void_p), ("ld_pre", _i64)]


class GemmDesc(ctypes.Structure):
    """Mirror of ``mg_gemm_desc`` (include/moegan_hip.h)."""
    _fields_ = [("M", _i32), ("N", _i32), ("K", _i32), ("A", _c_void_p), ("lda", _i64), ("B", _c_void_p),
                ("ldb", _i64), ("C", _c_void_p), ("ldc", _i64), ("ep", ctypes.POINTER(Epilogue))]


class PrepDesc(ctypes.Structure):
    """Mirror of ``mg_prep_desc``."""
    _fields_ = [("kind", _i32), ("Cout", _i32), ("Cin", _i32), ("KH", _i32), ("KW", _i32), ("rows", _i32),
                ("n", _i64), ("W", _c_void_p), ("aux", _c_void_p), ("aux2", _c_void_p), ("out", _c_void_p)]


class ColsumDesc(ctypes.Structure):
    """Mirror of ``mg_colsum_desc``."""
    _fields_ = [("dtype", _i32), ("R", _i32), ("C", _i32), ("ld", _i64), ("X", _c_void_p), ("out", _c_void_p)]


class WnDesc(ctypes.Structure):
    """Mirror of ``mg_wn_desc``."""
    _fields_ = [("O", _i32), ("K", _i32), ("v", _c_void_p), ("g", _c_void_p), ("norm", _c_void_p), ("W", _c_void_p),
                ("gW", _c_void_p), ("gv", _c_void_p), ("gg", _c_void_p)]


class RouterParamDesc(ctypes.Structure):
    """Mirror of ``mg_router_param_desc``."""
    _fields_ = [("mu", _c_void_p), ("rho", _c_void_p), ("eps", _c_void_p), ("gW", _c_void_p), ("kl_coef", _c_void_p),
                ("gmu", _c_void_p), ("grho", _c_void_p), ("n", _i64)]


class QuantDesc(ctypes.Structure):
    """Mirror of ``mg_quant_desc``."""
    _fields_ = [("x", _c_void_p), ("ldx", _i64), ("rows", _i64), ("K", _i32), ("q", _c_void_p), ("scale", _c_void_p)]


class GuardDesc(ctypes.Structure):
    """Mirror of ``mg_guard_desc``."""
    _fields_ = [("x", _c_void_p * 4), ("n", _i32 * 4), ("bit", _i32 * 4), ("nwin", _i32), ("reset_bits", _i32 * 2),
                ("keep_mask", _i32 * 2), ("bad_mask", _i32 * 2), ("set_bits", _i32 * 2)]


# Argument types are derived from include/moegan_hip.h itself, so the binding
# cannot drift from the C ABI (the header travels with the library).
_HEADER = os.path.abspath(os.path.join(_HERE, "..", "..", "include", "moegan_hip.h"))
_CTYPE = {"int": _i32, "int32_t": _i32, "int64_t": _i64, "uint64_t": ctypes.c_uint64, "size_t": ctypes.c_size_t,
          "float": _f32,
          "void": _c_void_p, "mg_epilogue": ctypes.POINTER(Epilogue), "mg_gemm_desc": ctypes.POINTER(GemmDesc),
          "mg_prep_desc": ctypes.POINTER(PrepDesc), "mg_colsum_desc": ctypes.POINTER(ColsumDesc),
          "mg_wn_desc": ctypes.POINTER(WnDesc), "mg_router_param_desc": ctypes.POINTER(RouterParamDesc),
          "mg_guard_desc": ctypes.POINTER(GuardDesc), "mg_quant_desc": ctypes.POINTER(QuantDesc)}
_RESTYPE = {"int": ctypes.c_int32, "int64_t": ctypes.c_int64, "const char*": ctypes.c_char_p}
SIG_RE = r"\b(int|int64_t|const char\*)\s+(mg_\w+)\(([^)]*)\);"


def _parse_header(path=_HEADER):
    """{name: (restype, [argtypes])} for every entry point declared in the C-ABI header."""
    import re
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    sigs = {}
    for ret, name, args in re.findall(SIG_RE, txt, flags=re.S):
        types, names = [], []
        for a in args.split(","):
            a = " ".join(a.split())
            if not a or a == "void":
                continue
            base = a.replace("const ", "").split()[0].rstrip("*")
            if "*" in a:
                types.append(_CTYPE[base] if base.endswith("_desc") or base == "mg_epilogue" else _c_void_p)
            else:
                types.append(_CTYPE[base])
            names.append(a.replace("*", " ").split()[-1])
        sigs[name] = (_RESTYPE[ret], types)
        ARGNAMES[name] = names
    return sigs


ARGNAMES = {}  # entry point -> parameter names, in order (the roofline attribution reads shapes by name)
_SIGS = _parse_header()
EP = ctypes.POINTER(Epilogue)

_lib = None


class MGError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MGError(f"libmoegan_hip.so not built ({LIB_PATH}); run __graft_entry__.build()")
        h = ctypes.CDLL(LIB_PATH)
        variant = bool(os.environ.get("MOEGAN_HIP_LIB"))  # an A/B build (tools/build_variants.sh) of older sources
        for name, (res, args) in _SIGS.items():
            if variant and not hasattr(h, name):
                continue  # an entry point newer than the variant: left unbound there
            fn = getattr(h, name)
            fn.argtypes = list(args)
            fn.restype = res
        _lib = h
        # A/B across processes (bench.py runs): MOEGAN_TUNE="slot=value,slot=value" sets library tuning slots at load
        for kv in filter(None, os.environ.get("MOEGAN_TUNE", "").split(",")):
            k, v = kv.split("=")
            if h.mg_set_tuning(int(k), int(v)) != 0:
                raise MGError(f"MOEGAN_TUNE {kv}: {h.mg_last_error().decode()}")
    return _lib


def source_hash_expected():
    """Hash of the HIP sources shipped next to the library (csrc/srchash.py)."""
    import importlib.util
    path = os.path.join(_HERE, "..", "csrc", "srchash.py")
    spec = importlib.util.spec_from_file_location("_mg_srchash", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.source_hash()


def check_source_hash():
    """Raise unless the loaded library was built from the sources in this tree."""
    got = lib().mg_source_hash().decode()
    want = source_hash_expected()
    if got != want:
        raise MGError(f"libmoegan_hip.so was built from other sources (hash {got}, tree {want}): rebuild it")
    return got


def exported_symbols():
    return list(_SIGS)


# Optional observer of every C-ABI call (moegan_mi/roofline.py): HOOK(name, args, run) must call run() once.
HOOK = None
# Optional live timer of one call signature (LiveTimer below; bench.py's roofline kernel)
LIVE = None


def scalar_signature(name, args):
    """(name, the call's integer / float arguments in order): the shape of a call, without its pointers."""
    types = _SIGS[name][1]
    vals = []
    for t, v in zip(types, args):
        if t in (_i32, _i64, _f32):
            vals.append(v.value if hasattr(v, "value") else v)
    return (name, tuple(vals))


class LiveTimer:
    """Times every call whose scalar_signature equals ``signature`` while ``active``: the call becomes an eager
    segment of a captured step (graphs.eager), bracketed by fence-free HIP events (mg_timer_event_*: a default
    event's system-scope release writes back and invalidates L2, which inflated the bracketed kernel by ~18 %) and,
    outside the events, by mg_mark begin / end kernels so a rocprofv3 trace of the same run finds the call's
    dispatches (tools/roofline_kernel.py).  Marks and events run whether or not ``active``, so every replay has the
    same dispatch sequence."""

    def __init__(self, signature, active=False):
        self.signature = signature
        self.active = active
        self.pairs = []

    def want(self, name, args):
        return name == self.signature[0] and scalar_signature(name, args) == self.signature

    def _event(self):
        h = ctypes.c_void_p()
        if lib().mg_timer_event_create(ctypes.addressof(h)) != 0:
            raise MGError(lib().mg_last_error().decode())
        return h

    def run(self, fn, args):
        from . import graphs

        # the call enqueues on the stream current when it runs: at a replay of a captured step that is the
        # stream the graphs replay on, not the capture stream its arguments were built on (the last parameter
        # of every entry point is the stream)
        names = ARGNAMES.get(fn.__name__, [])
        restream = bool(names) and names[-1] == "stream"

        def timed():
            st = stream()
            call_args = args[:-1] + (st,) if restream else args
            lib().mg_mark(0, st)
            s, e = (self._event(), self._event()) if self.active else (None, None)
            if s is not None:
                lib().mg_timer_event_record(s, st)
            rc = fn(*call_args)
            if e is not None:
                lib().mg_timer_event_record(e, st)
                self.pairs.append((s, e))
            lib().mg_mark(1, st)
            return rc
        return graphs.eager(timed)

    def results(self):
        """Per timed launch, its duration in ms (waits for the last event); releases the events."""
        out = []
        for s, e in self.pairs:
            ms = ctypes.c_float()
            if lib().mg_timer_event_elapsed(s, e, ctypes.addressof(ms)) != 0:
                raise MGError(lib().mg_last_error().decode())
            out.append(ms.value)
            lib().mg_timer_event_destroy(s)
            lib().mg_timer_event_destroy(e)
        self.pairs = []
        return out


def call(name, *args):
    fn = getattr(lib(), name)
    if LIVE is not None and LIVE.want(name, args):
        rc = LIVE.run(fn, args)
    else:
        rc = fn(*args) if HOOK is None else HOOK(name, args, lambda: fn(*args))
    if rc != 0:
        raise MGError(f"{name} failed ({rc}): {lib().mg_last_error().decode()}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dt(t):
    if t.dtype == torch.float32:
        return MG_F32
    if t.dtype == torch.bfloat16:
        return MG_BF16
    raise MGError(f"unsupported dtype {t.dtype}")


def epilogue(alpha=1.0, bias=None, scale=None, scale_shift=0, scale_ld=0, rowscale=None, act=0, aux=None,
             ld_aux=0, resid=None, ld_res=0, accumulate=0, atomic=0, remap_lgcin=0, remap_taps=0, a_idx=None,
             a_idx_div=1, a_rowscale=None, a_gelu=0, addvec=None, add_shift=0, add_ld=0, out_pre=None, ld_pre=0):
    e = Epilogue(alpha, ptr(bias), ptr(scale), scale_shift, scale_ld, ptr(rowscale), act, ptr(aux), ld_aux,
                 ptr(resid), ld_res, accumulate, atomic, remap_lgcin, remap_taps, ptr(a_idx), a_idx_div,
                 ptr(a_rowscale), a_gelu, ptr(addvec), add_shift, add_ld, ptr(out_pre), ld_pre)
    # keep the tensors alive until the launch has been enqueued
    e._keep = (bias, scale, rowscale, aux, resid, a_idx, a_rowscale, addvec, out_pre)
    return e
