"""ctypes wrappers over the oracle libraries (TEST / BASELINE INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
  * lib/libsks_oracle.so   — CPU restatement of the reference path (sks_oracle.cpp)
  * lib/libsks_refport.so  — reference-faithful port used as the CPU baseline
  * _ref/libref_fasta_ani.so — the reference's own fasta_processing.cpp and
    ani_estimation.cpp (built only where /root/reference exists)
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
REF_DIR = os.path.join(HERE, "_ref")


class OraBuf(C.Structure):
    _fields_ = [("data", C.c_void_p), ("lens", C.POINTER(C.c_uint64)),
                ("n", C.c_uint64), ("total", C.c_uint64)]


def build():
    """Compile the oracle (and oracle/_ref when the reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None
_rp = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(LIB_DIR, "libsks_oracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        u64p = C.POINTER(C.c_uint64)
        L.ora_buf_free.argtypes = [C.POINTER(OraBuf)]
        L.ora_fasta_records.argtypes = [C.c_char_p, C.POINTER(OraBuf)]
        L.ora_fasta_runs.argtypes = [C.c_char_p, C.POINTER(OraBuf)]
        L.ora_cut_runs.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(OraBuf)]
        L.ora_mask.argtypes = [C.c_int, C.c_int, C.c_uint64, u64p]
        L.ora_hash_bitset128.argtypes = [C.c_uint64, C.c_uint64, C.c_int]
        L.ora_hash_bitset128.restype = C.c_uint64
        L.ora_frac_min_hash.argtypes = [C.c_uint64] * 4 + [C.c_int, C.c_int64, C.c_int]
        L.ora_frac_min_hash.restype = C.c_uint64
        L.ora_windows.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, u64p,
                                  C.c_int64, C.c_int, C.POINTER(OraBuf)]
        L.ora_kmer_list.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, u64p,
                                    C.c_uint64, C.c_int64, C.c_int, C.POINTER(OraBuf)]
        L.ora_sketch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, u64p, C.c_int,
                                 C.c_uint64, C.c_int64, C.c_int, C.POINTER(OraBuf), u64p]
        L.ora_intersect.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]
        L.ora_intersect.restype = C.c_int32
        L.ora_containment.argtypes = [C.c_int, C.c_int]
        L.ora_containment.restype = C.c_double
        L.ora_binomial_estimator.argtypes = [C.c_double, C.c_int]
        L.ora_binomial_estimator.restype = C.c_double
        _lib = L
    return _lib


def _take_strings(b):
    lens = [int(b.lens[i]) for i in range(b.n)]
    raw = C.string_at(b.data, b.total) if b.total else b""
    out, o = [], 0
    for n in lens:
        out.append(raw[o:o + n])
        o += n
    return out


def fasta_records(path):
    b = OraBuf()
    rc = lib().ora_fasta_records(path.encode(), C.byref(b))
    if rc:
        raise FileNotFoundError(path)
    try:
        return _take_strings(b)
    finally:
        lib().ora_buf_free(C.byref(b))


def fasta_runs(path):
    b = OraBuf()
    rc = lib().ora_fasta_runs(path.encode(), C.byref(b))
    if rc:
        raise FileNotFoundError(path)
    try:
        return _take_strings(b)
    finally:
        lib().ora_buf_free(C.byref(b))


def cut_runs(data: bytes):
    b = OraBuf()
    buf = C.create_string_buffer(data, len(data))
    lib().ora_cut_runs(buf, len(data), C.byref(b))
    try:
        return _take_strings(b)
    finally:
        lib().ora_buf_free(C.byref(b))


def mask(w, k, seed=0):
    out = (C.c_uint64 * 2)()
    if lib().ora_mask(w, k, seed, out):
        raise ValueError("bad (w, k)")
    return int(out[0]) | (int(out[1]) << 64)


def hash_bitset128(value, flavour=0):
    return int(lib().ora_hash_bitset128(value & (2**64 - 1), value >> 64, flavour))


def frac_min_hash(c, m, w, nonce=1, flavour=0):
    return int(lib().ora_frac_min_hash(c & (2**64 - 1), c >> 64, m & (2**64 - 1), m >> 64,
                                       w, nonce, flavour))


def _runs_arrays(runs):
    codes = np.frombuffer(b"".join(runs), dtype=np.uint8) if runs else np.zeros(0, np.uint8)
    lens = np.array([len(r) for r in runs], dtype=np.uint64)
    return np.ascontiguousarray(codes), lens


def _mask_arr(m):
    return (C.c_uint64 * 2)(m & (2**64 - 1), m >> 64)


def windows(runs, w, m, nonce=1, flavour=0):
    """Per-window rows: F, R, C (python ints), H(C), fmh, run, offset."""
    codes, lens = _runs_arrays(runs)
    b = OraBuf()
    rc = lib().ora_windows(codes.ctypes.data, lens.ctypes.data, len(lens), w, _mask_arr(m),
                           nonce, flavour, C.byref(b))
    if rc:
        raise ValueError("bad w")
    try:
        a = np.ctypeslib.as_array(C.cast(b.data, C.POINTER(C.c_uint64)), shape=(b.total,)).copy() \
            if b.total else np.zeros(0, np.uint64)
    finally:
        lib().ora_buf_free(C.byref(b))
    return a.reshape(-1, 10)


def kmer_list(runs, w, m, c=200, nonce=1, flavour=0):
    """nucleotide_string_list_to_kmers with fmh % c == 0: rows of
    kmer_bits lo, hi, masked lo, hi, run, offset (uint64, shape (n, 6))."""
    codes, lens = _runs_arrays(runs)
    b = OraBuf()
    rc = lib().ora_kmer_list(codes.ctypes.data, lens.ctypes.data, len(lens), w, _mask_arr(m), c,
                             nonce, flavour, C.byref(b))
    if rc:
        raise ValueError("bad args")
    try:
        a = np.ctypeslib.as_array(C.cast(b.data, C.POINTER(C.c_uint64)), shape=(b.total,)).copy() \
            if b.total else np.zeros(0, np.uint64)
    finally:
        lib().ora_buf_free(C.byref(b))
    return a.reshape(-1, 6)


def sketch(runs, w, m, kind="frac", param=200, nonce=1, flavour=0):
    """Sorted unique canonical k-mers (uint64 array of shape (n, 2) = lo, hi) + windows."""
    codes, lens = _runs_arrays(runs)
    b = OraBuf()
    nw = C.c_uint64()
    rc = lib().ora_sketch(codes.ctypes.data, lens.ctypes.data, len(lens), w, _mask_arr(m),
                          0 if kind == "frac" else 1, param, nonce, flavour, C.byref(b),
                          C.byref(nw))
    if rc:
        raise ValueError("bad args")
    try:
        a = np.ctypeslib.as_array(C.cast(b.data, C.POINTER(C.c_uint64)), shape=(b.total,)).copy() \
            if b.total else np.zeros(0, np.uint64)
    finally:
        lib().ora_buf_free(C.byref(b))
    return a.reshape(-1, 2), int(nw.value)


def intersect(a, b):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    return int(lib().ora_intersect(a.ctypes.data, len(a), b.ctypes.data, len(b)))


def containment(inter, size):
    return float(lib().ora_containment(inter, size))


def binomial_estimator(c, k):
    return float(lib().ora_binomial_estimator(c, k))


# ---- reference-faithful port (CPU baseline) ------------------------------------
def refport():
    global _rp
    if _rp is None:
        path = os.path.join(LIB_DIR, "libsks_refport.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        u64p = C.POINTER(C.c_uint64)
        L.rp_set_flavour.argtypes = [C.c_int]
        L.rp_sketch_runs.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, u64p,
                                     C.c_uint64, C.c_int64]
        L.rp_sketch_runs.restype = C.c_void_p
        L.rp_bottom_runs.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, u64p,
                                     C.c_uint64, C.c_int64]
        L.rp_bottom_runs.restype = C.c_void_p
        L.rp_sketch_files.argtypes = [C.POINTER(C.c_char_p), C.c_int, C.c_int, u64p, C.c_uint64,
                                      C.c_int64, C.c_int, C.POINTER(C.c_void_p)]
        L.rp_set_from_elems.argtypes = [C.c_void_p, C.c_uint64, C.c_int, u64p]
        L.rp_set_from_elems.restype = C.c_void_p
        L.rp_set_size.argtypes = [C.c_void_p]
        L.rp_set_size.restype = C.c_uint64
        L.rp_set_dump.argtypes = [C.c_void_p, C.c_void_p]
        L.rp_set_free.argtypes = [C.c_void_p]
        L.rp_all_pairs.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_void_p]
        L.rp_pairs_prefix.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int64, C.c_int,
                                      C.c_void_p]
        _rp = L
    return _rp


class RefPortSet:
    def __init__(self, handle):
        self.h = handle

    def size(self):
        return int(refport().rp_set_size(self.h))

    def elems(self):
        n = self.size()
        out = np.zeros((n, 2), dtype=np.uint64)
        refport().rp_set_dump(self.h, out.ctypes.data)
        return out

    def __del__(self):
        if getattr(self, "h", None) and _rp is not None:
            _rp.rp_set_free(self.h)
            self.h = None


def refport_sketch_runs(runs, w, m, c=200, nonce=1, flavour=0):
    refport().rp_set_flavour(flavour)
    codes, lens = _runs_arrays(runs)
    return RefPortSet(refport().rp_sketch_runs(codes.ctypes.data, lens.ctypes.data, len(lens),
                                               w, _mask_arr(m), c, nonce))


def refport_sketch_codes(codes, lens, w, m, c=200, nonce=1, flavour=0):
    refport().rp_set_flavour(flavour)
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    return RefPortSet(refport().rp_sketch_runs(codes.ctypes.data, lens.ctypes.data, len(lens),
                                               w, _mask_arr(m), c, nonce))


def refport_bottom_codes(codes, lens, w, m, s, nonce=1, flavour=0):
    """Reference-style bottom-s (ref_port.cpp bottom_runs): the s distinct k-mers
    with the smallest (fmh, k-mer)."""
    refport().rp_set_flavour(flavour)
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    return RefPortSet(refport().rp_bottom_runs(codes.ctypes.data, lens.ctypes.data, len(lens),
                                               w, _mask_arr(m), s, nonce))


def refport_set_from_elems(elems, w, m):
    elems = np.ascontiguousarray(elems, dtype=np.uint64).reshape(-1, 2)
    return RefPortSet(refport().rp_set_from_elems(elems.ctypes.data, len(elems), w, _mask_arr(m)))


def refport_all_pairs(sets, threads=1):
    n = len(sets)
    arr = (C.c_void_p * n)(*[s.h for s in sets])
    out = np.zeros(n * n, dtype=np.int32)
    refport().rp_all_pairs(arr, n, threads, out.ctypes.data)
    return out.reshape(n, n)


def refport_pairs_prefix(sets, n_pairs, threads=1):
    n = len(sets)
    arr = (C.c_void_p * n)(*[s.h for s in sets])
    out = np.zeros(n_pairs, dtype=np.int32)
    refport().rp_pairs_prefix(arr, n, n_pairs, threads, out.ctypes.data)
    return out


# ---- the reference's own ingress / ANI (oracle/_ref) -----------------------------
def ref_available():
    return os.path.exists(os.path.join(REF_DIR, "libref_fasta_ani.so"))


def ref():
    global _ref
    if _ref is None:
        L = C.CDLL(os.path.join(REF_DIR, "libref_fasta_ani.so"))
        L.refx_buf_free.argtypes = [C.POINTER(OraBuf)]
        L.refx_fasta_records.argtypes = [C.c_char_p, C.POINTER(OraBuf)]
        L.refx_fasta_runs.argtypes = [C.c_char_p, C.POINTER(OraBuf)]
        L.refx_containment.argtypes = [C.c_int, C.c_int]
        L.refx_containment.restype = C.c_double
        L.refx_binomial_estimator.argtypes = [C.c_double, C.c_int]
        L.refx_binomial_estimator.restype = C.c_double
        _ref = L
    return _ref


def ref_fasta_records(path):
    b = OraBuf()
    ref().refx_fasta_records(path.encode(), C.byref(b))
    try:
        return _take_strings(b)
    finally:
        ref().refx_buf_free(C.byref(b))


def ref_fasta_runs(path):
    b = OraBuf()
    ref().refx_fasta_runs(path.encode(), C.byref(b))
    try:
        return _take_strings(b)
    finally:
        ref().refx_buf_free(C.byref(b))
