"""ctypes binding of libsks.so (include/sks.h) for the tests and bench.py.

This is plumbing only: every computation happens in libsks.so (HIP kernels for
gfx950 + host ingress).  There is deliberately no CPU fallback — if the library
or a GPU is missing, the calls below raise.  Device buffers are torch tensors
on `cuda:N` whose data_ptr() is handed to the C ABI.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SKS_LIB") or os.path.join(PKG_DIR, "lib", "libsks.so")

SKS_FRAC_MOD = 0
SKS_BOTTOM_S = 1
INTERSECT_AUTO, INTERSECT_MERGE, INTERSECT_JOIN, INTERSECT_GLOBAL = 0, 1, 2, 3
FLAVOUR_BOOST_MIX = 0
FLAVOUR_BOOST_LEGACY = 1


# sks_status (include/sks.h)
SKS_OK, SKS_E_ARG, SKS_E_HIP, SKS_E_IO, SKS_E_NOMEM, SKS_E_UNSUPPORTED, SKS_E_LENGTH = range(7)


class SksError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sks error {code}: {msg}")
        self.code = code


class Policy(C.Structure):
    _fields_ = [("kind", C.c_int32), ("flavour", C.c_int32), ("param", C.c_uint64),
                ("nonce", C.c_int64)]


class SketchInfo(C.Structure):
    _fields_ = [("window", C.c_int32), ("elem_words", C.c_int32), ("mask", C.c_uint64 * 2),
                ("policy", Policy), ("n", C.c_uint32), ("has_names", C.c_int32)]


class Timings(C.Structure):
    _fields_ = [("scan_ms", C.c_float), ("post_ms", C.c_float), ("total_ms", C.c_float),
                ("windows", C.c_uint64), ("scan_launches", C.c_uint64),
                ("survivors", C.c_uint64)]


EXPORTED = [
    "sks_abi_version", "sks_last_error", "sks_build_info", "sks_mask_generate", "sks_mask_contiguous",
    "sks_frac_min_hash", "sks_containment", "sks_binomial_estimator", "sks_ani_from_counts",
    "sks_fasta_open", "sks_fasta_close", "sks_fasta_num_records", "sks_fasta_record",
    "sks_fasta_stream", "sks_fasta_stream_bytes", "sks_fasta_runs", "sks_ctx_create",
    "sks_ctx_destroy", "sks_ctx_set_stream", "sks_ctx_synchronize", "sks_ctx_last_timings",
    "sks_sketch_build", "sks_sketch_set_free", "sks_sketch_set_free_on_stream", "sks_sketch_set_num", "sks_sketch_set_elem_words",
    "sks_ctx_set_layout_blocks_hint", "sks_ctx_ani_table",
    "sks_sketch_set_sizes", "sks_sketch_set_windows", "sks_sketch_set_device_data",
    "sks_sketch_set_device_starts", "sks_sketch_set_device_sizes", "sks_sketch_set_starts",
    "sks_sketch_set_copy", "sks_sketch_set_export", "sks_intersect_pairs", "sks_intersect_all",
    "sks_synth_bases", "sks_intersect_sym", "sks_intersect_sym_tiles",
    "sks_ctx_last_intersect_ms", "sks_ctx_set_scan_grid", "sks_ctx_set_intersect_kernel", "sks_join_layout_log_b", "sks_sketch_union", "sks_sketch_union_wide",
    "sks_join_layout_capacity", "sks_join_layout_build", "sks_intersect_sym_layout", "sks_fasta_parse_device",
    "sks_ctx_last_ingress_ms", "sks_kmer_list_build", "sks_kmer_list_free", "sks_kmer_list_total",
    "sks_kmer_list_counts", "sks_kmer_list_device_positions", "sks_kmer_list_device_bits",
    "sks_kmer_list_copy", "sks_ctx_device", "sks_sketch_set_info", "sks_sketch_set_set_names",
    "sks_sketch_set_name", "sks_sketch_set_save", "sks_sketch_set_load", "sks_sketch_set_concat",
    "sks_intersect_layout_tiles",
    "sks_join_layout_bounds", "sks_join_layout_groups", "sks_join_layout_boff_words",
    "sks_ctx_set_join_check", "sks_ctx_join_check_violations", "sks_intersect_layout_pair_tiles",
    "sks_sketch_set_export_csr", "sks_ani_matrix", "sks_ani_rows", "sks_ani_tiles",
    "sks_intersect_layout_ani", "sks_host_alloc", "sks_host_free", "sks_join_layout_stat_copy",
    "sks_sketches_export", "sks_all_pairs_ani", "sks_windows_dense", "sks_windows_dense_row_words",
    "sks_join_layout_bounds_for_mask", "sks_layout_tiles_ani",
]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libsks.so not built ({LIB_PATH}); run __graft_entry__.build()")
    # PyTorch-ROCm ships its own libamdhip64 with the same SONAME as /opt/rocm's
    # (libamdhip64.so.7): whichever loads first serves both.  Load torch first
    # when it is installed, so a process that also uses torch device memory and
    # streams runs ONE HIP runtime — the order every GPU test and bench.py use.
    # (libsks loaded first, then torch, left sks_ctx_create without devices.)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    u64p = C.POINTER(C.c_uint64)
    vp = C.c_void_p
    L.sks_last_error.restype = C.c_char_p
    L.sks_build_info.restype = C.c_char_p
    L.sks_mask_generate.argtypes = [C.c_int, C.c_int, C.c_uint64, u64p]
    L.sks_mask_contiguous.argtypes = [C.c_int, u64p]
    L.sks_frac_min_hash.argtypes = [u64p, u64p, C.c_int, C.c_int64, C.c_int]
    L.sks_frac_min_hash.restype = C.c_uint64
    L.sks_containment.argtypes = [C.c_int, C.c_int]
    L.sks_containment.restype = C.c_double
    L.sks_binomial_estimator.argtypes = [C.c_double, C.c_int]
    L.sks_binomial_estimator.restype = C.c_double
    L.sks_ani_from_counts.argtypes = [vp, vp, C.c_uint64, C.c_int, vp, vp]
    L.sks_fasta_open.argtypes = [C.c_char_p, C.POINTER(vp)]
    L.sks_fasta_close.argtypes = [vp]
    L.sks_fasta_close.restype = None
    L.sks_fasta_num_records.argtypes = [vp]
    L.sks_fasta_num_records.restype = C.c_uint64
    L.sks_fasta_record.argtypes = [vp, C.c_uint64, C.POINTER(vp), u64p]
    L.sks_fasta_stream.argtypes = [vp]
    L.sks_fasta_stream.restype = vp
    L.sks_fasta_stream_bytes.argtypes = [vp]
    L.sks_fasta_stream_bytes.restype = C.c_uint64
    L.sks_fasta_runs.argtypes = [vp, vp, vp, u64p, u64p]
    L.sks_ctx_create.argtypes = [C.c_int, vp, C.POINTER(vp)]
    L.sks_ctx_destroy.argtypes = [vp]
    L.sks_ctx_set_stream.argtypes = [vp, vp]
    L.sks_ctx_synchronize.argtypes = [vp]
    L.sks_ctx_last_timings.argtypes = [vp, C.POINTER(Timings)]
    L.sks_ctx_set_scan_grid.argtypes = [vp, C.c_int]
    L.sks_ctx_set_intersect_kernel.argtypes = [vp, C.c_int]
    L.sks_sketch_union.argtypes = [vp, vp, C.c_uint64, vp, u64p]
    L.sks_sketch_union_wide.argtypes = [vp, vp, C.c_uint64, vp, u64p]
    L.sks_join_layout_log_b.argtypes = [C.c_uint32]
    L.sks_join_layout_log_b.restype = C.c_uint32
    L.sks_join_layout_capacity.argtypes = []
    L.sks_join_layout_capacity.restype = C.c_uint32
    L.sks_join_layout_build.argtypes = [vp, vp, vp, vp, C.c_int, C.c_uint32, C.c_uint64, C.c_uint32, vp,
                                        vp, vp, vp, vp, C.POINTER(C.c_uint32)]
    L.sks_join_layout_bounds.argtypes = [vp, vp, vp, vp, C.c_int, C.c_uint32, C.c_uint32, vp]
    L.sks_join_layout_groups.argtypes = [C.c_uint32]
    L.sks_join_layout_groups.restype = C.c_uint32
    L.sks_join_layout_boff_words.argtypes = [C.c_uint32]
    L.sks_join_layout_boff_words.restype = C.c_uint32
    L.sks_intersect_sym_layout.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_int, vp, vp, vp, vp, C.c_uint64,
                                           C.c_uint64, vp]
    L.sks_intersect_layout_tiles.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_int, vp, vp, vp, vp, C.c_uint32,
                                             vp, C.c_uint64, C.c_uint64, C.c_int, vp]
    L.sks_intersect_layout_pair_tiles.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_int, vp, vp, vp, vp,
                                                  C.c_uint32, vp, vp, vp, vp, C.c_uint32, vp, C.c_uint64,
                                                  C.c_uint64, C.c_int, vp]
    L.sks_intersect_layout_ani.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_int, vp, vp, vp, vp, C.c_uint32,
                                           vp, vp, vp, vp, C.c_uint32, vp, C.c_uint64, C.c_uint64, C.c_int, vp,
                                           vp, C.c_int, vp]
    L.sks_host_alloc.argtypes = [C.c_uint64, C.c_int, C.POINTER(vp)]
    L.sks_host_free.argtypes = [vp]
    L.sks_join_layout_stat_copy.argtypes = [vp, vp]
    L.sks_sketches_export.argtypes = [vp, vp, vp, vp, C.c_int, C.c_uint32, vp, C.c_uint64, vp]
    L.sks_all_pairs_ani.argtypes = [vp, vp, vp, vp, C.c_int, C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, vp, vp,
                                    vp]
    L.sks_layout_tiles_ani.argtypes = [vp, vp, vp, vp, C.c_int, C.c_uint32, C.c_uint64, C.c_uint32, vp,
                                       C.c_uint32, C.c_uint32, vp, C.c_uint64, C.c_uint32, vp, C.c_int, vp, vp, vp]
    L.sks_sketch_set_export_csr.argtypes = [vp, vp, vp]
    L.sks_ani_matrix.argtypes = [vp, vp, C.c_uint32, C.c_int, vp, vp]
    L.sks_ani_rows.argtypes = [vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, vp, vp]
    L.sks_ani_tiles.argtypes = [vp, vp, vp, C.c_uint64, C.c_uint32, vp, C.c_int, vp]
    L.sks_ctx_set_join_check.argtypes = [vp, C.c_int]
    L.sks_ctx_ani_table.argtypes = [vp, C.c_uint32, C.c_int]
    L.sks_ctx_join_check_violations.argtypes = [vp, u64p]
    L.sks_ctx_last_intersect_ms.argtypes = [vp, C.POINTER(C.c_float)]
    L.sks_ctx_last_ingress_ms.argtypes = [vp, C.POINTER(C.c_float)]
    L.sks_ctx_device.argtypes = [vp]
    L.sks_sketch_set_info.argtypes = [vp, C.POINTER(SketchInfo)]
    L.sks_sketch_set_set_names.argtypes = [vp, vp]
    L.sks_sketch_set_name.argtypes = [vp, C.c_uint32]
    L.sks_sketch_set_name.restype = C.c_char_p
    L.sks_sketch_set_save.argtypes = [vp, C.c_char_p]
    L.sks_sketch_set_load.argtypes = [vp, C.c_char_p, C.POINTER(vp)]
    L.sks_sketch_set_concat.argtypes = [vp, vp, C.c_uint32, C.POINTER(vp)]
    L.sks_kmer_list_build.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, C.c_int, u64p,
                                      C.POINTER(Policy), C.POINTER(vp)]
    L.sks_windows_dense.argtypes = [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, u64p, vp, vp]
    L.sks_windows_dense_row_words.argtypes = [C.c_int]
    L.sks_join_layout_bounds_for_mask.argtypes = [u64p, C.c_uint32, C.c_int, vp]
    L.sks_kmer_list_free.argtypes = [vp]
    L.sks_kmer_list_total.argtypes = [vp]
    L.sks_kmer_list_total.restype = C.c_uint64
    L.sks_kmer_list_counts.argtypes = [vp, vp]
    L.sks_kmer_list_copy.argtypes = [vp, vp, vp]
    for f in ("sks_kmer_list_device_positions", "sks_kmer_list_device_bits"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = vp
    L.sks_fasta_parse_device.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp, C.c_uint64,
                                         u64p, u64p]
    L.sks_sketch_build.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, C.c_int, u64p,
                                   C.POINTER(Policy), C.POINTER(vp)]
    L.sks_sketch_set_free.argtypes = [vp]
    L.sks_sketch_set_free_on_stream.argtypes = [vp, vp]
    L.sks_sketch_set_num.argtypes = [vp]
    L.sks_sketch_set_num.restype = C.c_uint32
    L.sks_sketch_set_elem_words.argtypes = [vp]
    L.sks_sketch_set_sizes.argtypes = [vp, vp]
    L.sks_sketch_set_windows.argtypes = [vp, vp]
    L.sks_sketch_set_starts.argtypes = [vp, vp]
    for f in ("sks_sketch_set_device_data", "sks_sketch_set_device_starts",
              "sks_sketch_set_device_sizes"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = vp
    L.sks_sketch_set_copy.argtypes = [vp, C.c_uint32, vp]
    L.sks_sketch_set_export.argtypes = [vp, vp, C.c_uint64, vp]
    L.sks_intersect_pairs.argtypes = [vp, vp, vp, vp, C.c_int, vp, vp, C.c_uint64, vp]
    L.sks_intersect_all.argtypes = [vp, vp, vp, vp, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                                    vp]
    L.sks_intersect_sym.argtypes = [vp, vp, vp, vp, C.c_int, C.c_uint32, C.c_uint64, C.c_uint64,
                                    vp]
    L.sks_intersect_sym_tiles.argtypes = [C.c_uint32]
    L.sks_intersect_sym_tiles.restype = C.c_uint64
    L.sks_synth_bases.argtypes = [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_double,
                                  C.c_uint64]
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise SksError(rc, lib().sks_last_error().decode(errors="replace"))


def _mask_arr(mask):
    return (C.c_uint64 * 2)(mask & (2**64 - 1), mask >> 64)


# ---- host helpers -------------------------------------------------------------------
def mask_generate(window, k, seed=0):
    out = (C.c_uint64 * 2)()
    check(lib().sks_mask_generate(window, k, seed, out))
    return int(out[0]) | (int(out[1]) << 64)


def mask_contiguous(length):
    out = (C.c_uint64 * 2)()
    check(lib().sks_mask_contiguous(length, out))
    return int(out[0]) | (int(out[1]) << 64)


def frac_min_hash(kmer, mask, window, nonce=1, flavour=0):
    return int(lib().sks_frac_min_hash(_mask_arr(kmer), _mask_arr(mask), window, nonce, flavour))


def join_layout_log_b(max_sketch_size):
    return int(lib().sks_join_layout_log_b(max_sketch_size))


def join_layout_capacity():
    return int(lib().sks_join_layout_capacity())


def join_layout_groups(log_b):
    return int(lib().sks_join_layout_groups(log_b))


def join_layout_bounds_for_mask(mask, log_b, elem_words=1):
    """sks_join_layout_bounds_for_mask: the mask-derived group bounds, a uint64 array
    of (join_layout_groups(log_b) + 1) * elem_words words (host)."""
    out = np.zeros((join_layout_groups(log_b) + 1) * elem_words, dtype=np.uint64)
    check(lib().sks_join_layout_bounds_for_mask(_mask_arr(mask), log_b, elem_words, out.ctypes.data))
    return out


def join_layout_boff_words(log_b):
    """u32 words of one block's boff row (2^log_b bucket starts + region ends)."""
    return int(lib().sks_join_layout_boff_words(log_b))


def intersect_sym_tiles(n):
    return int(lib().sks_intersect_sym_tiles(n))


def containment(inter, size):
    return float(lib().sks_containment(inter, size))


def binomial_estimator(c, k):
    return float(lib().sks_binomial_estimator(c, k))


def ani_from_counts(inter, size_first, k):
    inter = np.ascontiguousarray(inter, dtype=np.int32)
    size_first = np.ascontiguousarray(size_first, dtype=np.int32)
    cont = np.zeros(inter.shape, dtype=np.float64)
    ani = np.zeros(inter.shape, dtype=np.float64)
    check(lib().sks_ani_from_counts(inter.ctypes.data, size_first.ctypes.data, inter.size, k,
                                    cont.ctypes.data, ani.ctypes.data))
    return cont, ani


class Fasta:
    """sks_fasta_open: the reference's strings_from_fasta record rules."""

    def __init__(self, path):
        h = C.c_void_p()
        check(lib().sks_fasta_open(os.fsencode(path), C.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().sks_fasta_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def num_records(self):
        return int(lib().sks_fasta_num_records(self.h))

    def records(self):
        out = []
        for i in range(self.num_records()):
            p = C.c_void_p()
            n = C.c_uint64()
            check(lib().sks_fasta_record(self.h, i, C.byref(p), C.byref(n)))
            out.append(C.string_at(p, n.value) if n.value else b"")
        return out

    def stream(self):
        n = int(lib().sks_fasta_stream_bytes(self.h))
        if n == 0:
            return np.zeros(0, dtype=np.uint8)
        p = lib().sks_fasta_stream(self.h)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n,)).copy()

    def runs(self):
        nc, nr = C.c_uint64(0), C.c_uint64(0)
        check(lib().sks_fasta_runs(self.h, None, None, C.byref(nc), C.byref(nr)))
        codes = np.zeros(max(nc.value, 1), dtype=np.uint8)
        lens = np.zeros(max(nr.value, 1), dtype=np.uint64)
        check(lib().sks_fasta_runs(self.h, codes.ctypes.data, lens.ctypes.data, C.byref(nc),
                                   C.byref(nr)))
        codes, lens = codes[:nc.value], lens[:nr.value]
        out, o = [], 0
        for n in lens:
            out.append(codes[o:o + int(n)].tobytes())
            o += int(n)
        return out


class HostBuffer:
    """sks_host_alloc: pinned host memory mapped for the devices (the destination
    of sks_intersect_layout_ani), coherent (fine-grained) or not; .array is a
    numpy view of it."""

    def __init__(self, nbytes, dtype=np.float64, coherent=False):
        p = C.c_void_p()
        check(lib().sks_host_alloc(int(nbytes), 1 if coherent else 0, C.byref(p)))
        self.ptr = int(p.value or 0)
        self.nbytes = int(nbytes)
        n = self.nbytes // np.dtype(dtype).itemsize
        self.array = (np.ctypeslib.as_array(C.cast(self.ptr, C.POINTER(C.c_uint8)), shape=(self.nbytes,))
                      .view(dtype)[:n] if self.ptr else np.zeros(0, dtype=dtype))

    def free(self):
        if self.ptr:
            self.array = None
            check(lib().sks_host_free(C.c_void_p(self.ptr)))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---- device ---------------------------------------------------------------------------------
class Context:
    def __init__(self, device=0, stream=None):
        h = C.c_void_p()
        check(lib().sks_ctx_create(device, C.c_void_p(stream) if stream else None, C.byref(h)))
        self.h = h
        self.device = device
        self.stream = stream or 0  # hipStream_t handle the context's work is queued on (0: null)

    def set_stream(self, stream):
        check(lib().sks_ctx_set_stream(self.h, C.c_void_p(stream) if stream else None))
        self.stream = stream or 0

    def set_scan_grid(self, grid):
        check(lib().sks_ctx_set_scan_grid(self.h, grid))

    def sketch_union(self, d_in, n, d_out, elem_words=1):
        """sks_sketch_union (elem_words 1: u64 values) or sks_sketch_union_wide
        (elem_words 2: n (lo, hi) pairs): sorted distinct k-mers of d_in into d_out;
        returns the count."""
        k = C.c_uint64(0)
        fn = lib().sks_sketch_union if elem_words == 1 else lib().sks_sketch_union_wide
        check(fn(self.h, C.c_void_p(d_in), n, C.c_void_p(d_out), C.byref(k)))
        return int(k.value)

    def join_layout_build(self, data_ptr, starts_ptr, sizes_ptr, n, log_b, out_vals, out_masks,
                          out_boff, out_bstart, stat=True, total=None, bounds=None, elem_words=1):
        """sks_join_layout_build; returns the largest block-bucket population
        (entries; 2**32 - 1: layout invalid), or None with stat=False (no
        read-back).  total: the sizes' sum when known (with stat=False the call
        then does not wait for the stream at all); bounds: device pointer of the
        group bounds (None: the set's own)."""
        mx = C.c_uint32(0)
        check(lib().sks_join_layout_build(self.h, C.c_void_p(data_ptr), C.c_void_p(starts_ptr),
                                          C.c_void_p(sizes_ptr), elem_words, n,
                                          (1 << 64) - 1 if total is None else int(total), log_b,
                                          C.c_void_p(bounds) if bounds else None,
                                          C.c_void_p(out_vals), C.c_void_p(out_masks), C.c_void_p(out_boff),
                                          C.c_void_p(out_bstart), C.byref(mx) if stat else None))
        return mx.value if stat else None

    def set_layout_blocks_hint(self, blocks):
        """sks_ctx_set_layout_blocks_hint: blocks that hold sketches in the next layout builds (0: all)."""
        check(lib().sks_ctx_set_layout_blocks_hint(self.h, C.c_uint32(int(blocks))))

    def ani_table(self, size, kmer_num_ones):
        """sks_ctx_ani_table: ANI by shared-element count for sets of `size` elements (fused ANI reads it)."""
        check(lib().sks_ctx_ani_table(self.h, C.c_uint32(int(size)), int(kmer_num_ones)))

    def all_pairs_ani(self, data, starts, sizes, n, max_size, total, kmer_num_ones, ani, counts, status,
                      elem_words=1):
        """sks_all_pairs_ani (device pointers; ani: device or pinned host pointer, or 0
        for counts only; counts / status may be 0)."""
        check(lib().sks_all_pairs_ani(self.h, C.c_void_p(data), C.c_void_p(starts), C.c_void_p(sizes), elem_words,
                                      n, max_size, total, kmer_num_ones, C.c_void_p(ani) if ani else None,
                                      C.c_void_p(counts) if counts else None, C.c_void_p(status) if status else None))

    def layout_tiles_ani(self, data, starts, sizes, n, total, log_b, bounds, blocks_hint, blk0, tiles, n_tiles,
                         n_global, sizes_global, kmer_num_ones, ani, counts, status, elem_words=1):
        """sks_layout_tiles_ani (device pointers; ani: device or pinned host pointer,
        or 0 for counts only): layout + join of a global tile list in one call."""
        v = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        check(lib().sks_layout_tiles_ani(self.h, v(data), v(starts), v(sizes), elem_words, n, total, log_b,
                                         v(bounds), blocks_hint, blk0, v(tiles), n_tiles, n_global,
                                         v(sizes_global), kmer_num_ones, v(ani), v(counts), v(status)))

    def sketches_export(self, data, starts, sizes, n, dst, stride, dst_sizes, elem_words=1):
        """sks_sketches_export (device pointers): sketches padded to a fixed stride."""
        check(lib().sks_sketches_export(self.h, C.c_void_p(data), C.c_void_p(starts), C.c_void_p(sizes), elem_words,
                                        n, C.c_void_p(dst), stride, C.c_void_p(dst_sizes)))

    def join_layout_stat_copy(self, d_dst):
        """sks_join_layout_stat_copy: the last build's (max block bucket, invalid)
        words into the device buffer d_dst (2 x u32), queued on the stream."""
        check(lib().sks_join_layout_stat_copy(self.h, C.c_void_p(d_dst)))

    def join_layout_bounds(self, data_ptr, starts_ptr, sizes_ptr, n, log_b, out_bounds, elem_words=1):
        """sks_join_layout_bounds: the set's group bounds (device pointer out_bounds,
        (join_layout_groups(log_b) + 1) * elem_words words)."""
        check(lib().sks_join_layout_bounds(self.h, C.c_void_p(data_ptr), C.c_void_p(starts_ptr),
                                           C.c_void_p(sizes_ptr), elem_words, n, log_b, C.c_void_p(out_bounds)))

    def intersect_sym_layout(self, n, log_b, vals, masks, boff, bstart, tile_begin, tile_end, out,
                             elem_words=1):
        check(lib().sks_intersect_sym_layout(self.h, n, log_b, elem_words, C.c_void_p(vals), C.c_void_p(masks),
                                             C.c_void_p(boff), C.c_void_p(bstart), tile_begin,
                                             tile_end, C.c_void_p(out)))

    def intersect_layout_tiles(self, n, log_b, vals, masks, boff, bstart, blk0, tiles, tile_begin, tile_end,
                               packed, out, elem_words=1):
        """sks_intersect_layout_tiles: join tiles over a layout whose block 0 is
        global block blk0; counts ADDED to `out` (n x n both halves, or packed
        [tile][64][64]); tiles: device pointer of (I, J) u32 pairs, or 0."""
        check(lib().sks_intersect_layout_tiles(self.h, n, log_b, elem_words, C.c_void_p(vals), C.c_void_p(masks),
                                               C.c_void_p(boff), C.c_void_p(bstart), blk0,
                                               C.c_void_p(tiles) if tiles else None, tile_begin, tile_end,
                                               1 if packed else 0, C.c_void_p(out)))

    def intersect_layout_pair_tiles(self, n, log_b, rows, r_blk0, cols, c_blk0, tiles, tile_begin, tile_end,
                                    packed, out, elem_words=1):
        """sks_intersect_layout_pair_tiles: rows / cols are (vals, masks, boff, bstart)
        device pointers of two layouts; tiles: device pointer of (I, J) u32 pairs."""
        check(lib().sks_intersect_layout_pair_tiles(self.h, n, log_b, elem_words,
                                                    *(C.c_void_p(p) for p in rows), r_blk0,
                                                    *(C.c_void_p(p) for p in cols), c_blk0, C.c_void_p(tiles),
                                                    tile_begin, tile_end, 1 if packed else 0, C.c_void_p(out)))

    def intersect_layout_ani(self, n, log_b, rows, r_blk0, cols, c_blk0, tiles, tile_begin, tile_end, packed,
                             out, sizes, kmer_num_ones, ani, elem_words=1):
        """sks_intersect_layout_ani: intersect_layout_pair_tiles (tiles = 0: the
        upper-triangle range of one layout) plus the ANI of every counted pair,
        written by the join itself into `ani` (n * n float64; a device pointer or
        pinned host memory from HostBuffer); sizes: device int32 |S_i|."""
        check(lib().sks_intersect_layout_ani(self.h, n, log_b, elem_words, *(C.c_void_p(p) for p in rows), r_blk0,
                                             *(C.c_void_p(p) for p in cols), c_blk0,
                                             C.c_void_p(tiles) if tiles else None, tile_begin, tile_end,
                                             1 if packed else 0, C.c_void_p(out), C.c_void_p(sizes),
                                             kmer_num_ones, C.c_void_p(ani)))

    def ani_matrix(self, counts, n, kmer_num_ones, ani, cont=None):
        """sks_ani_matrix (device pointers): ANI of every ordered pair of the n x n counts."""
        check(lib().sks_ani_matrix(self.h, C.c_void_p(counts), n, kmer_num_ones,
                                   C.c_void_p(cont) if cont else None, C.c_void_p(ani)))

    def ani_rows(self, counts, n, row_begin, row_end, kmer_num_ones, ani, cont=None):
        """sks_ani_rows (device pointers): rows [row_begin, row_end) of ani_matrix."""
        check(lib().sks_ani_rows(self.h, C.c_void_p(counts), n, row_begin, row_end, kmer_num_ones,
                                 C.c_void_p(cont) if cont else None, C.c_void_p(ani)))

    def ani_tiles(self, packed, tiles, n_tiles, n, sizes, kmer_num_ones, ani):
        """sks_ani_tiles (device pointers): both orientations of every pair of packed tiles."""
        check(lib().sks_ani_tiles(self.h, C.c_void_p(packed), C.c_void_p(tiles), n_tiles, n, C.c_void_p(sizes),
                                  kmer_num_ones, C.c_void_p(ani)))

    def set_join_check(self, on):
        """sks_ctx_set_join_check: instrumented layout / join kernels (diagnostics)."""
        check(lib().sks_ctx_set_join_check(self.h, 1 if on else 0))

    def join_check_violations(self):
        v = C.c_uint64(0)
        check(lib().sks_ctx_join_check_violations(self.h, C.byref(v)))
        return int(v.value)

    def set_intersect_kernel(self, kind):
        """INTERSECT_AUTO / _MERGE / _JOIN / _GLOBAL (sks.h); all give identical counts."""
        check(lib().sks_ctx_set_intersect_kernel(self.h, kind))
        self._intersect_kernel = kind

    def synchronize(self):
        check(lib().sks_ctx_synchronize(self.h))

    def timings(self):
        t = Timings()
        check(lib().sks_ctx_last_timings(self.h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in Timings._fields_}

    def last_intersect_ms(self):
        ms = C.c_float()
        check(lib().sks_ctx_last_intersect_ms(self.h, C.byref(ms)))
        return float(ms.value)

    def last_ingress_ms(self):
        ms = C.c_float()
        check(lib().sks_ctx_last_ingress_ms(self.h, C.byref(ms)))
        return float(ms.value)

    def fasta_parse_device(self, d_raw_ptr, n_raw, d_stream_ptr=None, stream_cap=0,
                           d_rec_end_ptr=None, rec_cap=0):
        """Device strings_from_fasta; returns (stream_bytes, n_records)."""
        nb, nr = C.c_uint64(), C.c_uint64()
        check(lib().sks_fasta_parse_device(self.h, C.c_void_p(d_raw_ptr), n_raw,
                                           C.c_void_p(d_stream_ptr), stream_cap,
                                           C.c_void_p(d_rec_end_ptr), rec_cap, C.byref(nb),
                                           C.byref(nr)))
        return int(nb.value), int(nr.value)

    def close(self):
        if self.h:
            lib().sks_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sketch_build(self, d_seq_ptr, n_bytes, seg_off, window, mask, kind=SKS_FRAC_MOD,
                     param=200, nonce=1, flavour=0):
        seg = np.ascontiguousarray(seg_off, dtype=np.uint64)
        pol = Policy(kind, flavour, param, nonce)
        h = C.c_void_p()
        check(lib().sks_sketch_build(self.h, C.c_void_p(d_seq_ptr), n_bytes, seg.ctypes.data,
                                     len(seg) - 1, window, _mask_arr(mask), C.byref(pol),
                                     C.byref(h)))
        return SketchSet(h)

    def kmer_list(self, d_seq_ptr, n_bytes, seg_off, window, mask, c=200, nonce=1, flavour=0):
        """nucleotide_string_list_to_kmers on the device: returns (positions,
        bits[n, 4] = kmer_bits lo, hi, masked lo, hi, counts per segment)."""
        seg = np.ascontiguousarray(seg_off, dtype=np.uint64)
        pol = Policy(SKS_FRAC_MOD, flavour, c, nonce)
        h = C.c_void_p()
        check(lib().sks_kmer_list_build(self.h, C.c_void_p(d_seq_ptr), n_bytes, seg.ctypes.data,
                                        len(seg) - 1, window, _mask_arr(mask), C.byref(pol),
                                        C.byref(h)))
        try:
            n = int(lib().sks_kmer_list_total(h))
            pos = np.zeros(max(n, 1), np.uint64)
            bits = np.zeros(max(4 * n, 1), np.uint64)
            counts = np.zeros(max(len(seg) - 1, 1), np.uint64)
            check(lib().sks_kmer_list_copy(h, pos.ctypes.data, bits.ctypes.data))
            check(lib().sks_kmer_list_counts(h, counts.ctypes.data))
        finally:
            lib().sks_kmer_list_free(h)
        return pos[:n], bits[:4 * n].reshape(n, 4), counts[:len(seg) - 1]

    def windows_dense(self, d_seq_ptr, n_bytes, first, n_windows, window, mask, d_rows, d_valid):
        """sks_windows_dense (device pointers; queued on the context stream): every
        window starting in [first, first + n_windows) of the piece, dense by start."""
        check(lib().sks_windows_dense(self.h, C.c_void_p(d_seq_ptr), C.c_uint64(n_bytes), C.c_uint64(first),
                                      C.c_uint64(n_windows), window, _mask_arr(mask), C.c_void_p(d_rows),
                                      C.c_void_p(d_valid)))

    def load_sketches(self, path):
        h = C.c_void_p()
        check(lib().sks_sketch_set_load(self.h, str(path).encode(), C.byref(h)))
        return SketchSet(h)

    def concat(self, sets):
        arr = (C.c_void_p * len(sets))(*[s.h for s in sets])
        h = C.c_void_p()
        check(lib().sks_sketch_set_concat(self.h, arr, len(sets), C.byref(h)))
        return SketchSet(h)

    def intersect_pairs(self, data_ptr, starts_ptr, sizes_ptr, elem_words, a_ptr, b_ptr,
                        n_pairs, out_ptr):
        check(lib().sks_intersect_pairs(self.h, data_ptr, starts_ptr, sizes_ptr, elem_words,
                                        a_ptr, b_ptr, n_pairs, out_ptr))

    def intersect_all(self, data_ptr, starts_ptr, sizes_ptr, elem_words, n, row_begin, row_end,
                      out_ptr):
        check(lib().sks_intersect_all(self.h, data_ptr, starts_ptr, sizes_ptr, elem_words, n,
                                      row_begin, row_end, out_ptr))

    def intersect_sym(self, data_ptr, starts_ptr, sizes_ptr, elem_words, n, tile_begin, tile_end,
                      out_ptr):
        check(lib().sks_intersect_sym(self.h, data_ptr, starts_ptr, sizes_ptr, elem_words, n,
                                      tile_begin, tile_end, out_ptr))

    def synth_bases(self, d_out_ptr, n, seed, mut_seed=0, mut_rate=0.0, pos_offset=0):
        check(lib().sks_synth_bases(self.h, C.c_void_p(d_out_ptr), n, seed, mut_seed, mut_rate,
                                    pos_offset))


class _DeviceArray:
    """A device buffer described by __cuda_array_interface__ (torch.as_tensor
    wraps it without a copy)."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr,
                                         "data": (int(ptr), False), "version": 3, "strides": None}


class SketchSet:
    def __init__(self, h):
        self.h = h
        self.n = int(lib().sks_sketch_set_num(h))
        self.elem_words = int(lib().sks_sketch_set_elem_words(h))

    def free(self, stream=None):
        """sks_sketch_set_free, or with `stream` (a hipStream_t handle, e.g.
        torch.cuda.Stream().cuda_stream) sks_sketch_set_free_on_stream: no
        device-wide wait; every use of the set must be ordered on that stream."""
        if self.h:
            if stream is None:
                lib().sks_sketch_set_free(self.h)
            else:
                lib().sks_sketch_set_free_on_stream(self.h, C.c_void_p(stream))
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def info(self):
        i = SketchInfo()
        check(lib().sks_sketch_set_info(self.h, C.byref(i)))
        return {"window": i.window, "elem_words": i.elem_words,
                "mask": int(i.mask[0]) | int(i.mask[1]) << 64, "kind": i.policy.kind,
                "flavour": i.policy.flavour, "param": i.policy.param, "nonce": i.policy.nonce,
                "n": i.n, "has_names": bool(i.has_names)}

    def set_names(self, names):
        if names is None:
            check(lib().sks_sketch_set_set_names(self.h, None))
            return
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        check(lib().sks_sketch_set_set_names(self.h, arr))

    def names(self):
        out = []
        for i in range(self.n):
            v = lib().sks_sketch_set_name(self.h, i)
            if v is None:
                return None
            out.append(v.decode())
        return out

    def save(self, path):
        check(lib().sks_sketch_set_save(self.h, str(path).encode()))

    def sizes(self):
        out = np.zeros(max(self.n, 1), dtype=np.uint32)
        check(lib().sks_sketch_set_sizes(self.h, out.ctypes.data))
        return out[:self.n]

    def windows(self):
        out = np.zeros(max(self.n, 1), dtype=np.uint64)
        check(lib().sks_sketch_set_windows(self.h, out.ctypes.data))
        return out[:self.n]

    def starts(self):
        out = np.zeros(max(self.n, 1), dtype=np.uint64)
        check(lib().sks_sketch_set_starts(self.h, out.ctypes.data))
        return out[:self.n]

    def sketch(self, i):
        """Sketch i as a uint64 array of shape (size, 2) = (lo, hi)."""
        n = int(self.sizes()[i])
        buf = np.zeros(max(n * self.elem_words, 1), dtype=np.uint64)
        check(lib().sks_sketch_set_copy(self.h, i, buf.ctypes.data))
        buf = buf[:n * self.elem_words]
        if self.elem_words == 1:
            return np.stack([buf, np.zeros_like(buf)], axis=1)
        return buf.reshape(-1, 2)

    def copy_into(self, i, host_ptr):
        """Sketch i (size * elem_words u64) into caller memory (e.g. pinned); returns size."""
        check(lib().sks_sketch_set_copy(self.h, i, C.c_void_p(host_ptr)))
        return int(self.sizes()[i])

    def device_ptrs(self):
        L = lib()
        return (L.sks_sketch_set_device_data(self.h), L.sks_sketch_set_device_starts(self.h),
                L.sks_sketch_set_device_sizes(self.h))

    def device_tensors(self, device=0):
        """Zero-copy torch views of the set's device arrays: (data int64
        [total * elem_words], starts int64 [n], sizes int32 [n]).  The views do
        not keep the set alive: use them while the set is."""
        import torch
        d, st, sz = self.device_ptrs()
        total = int(self.sizes().astype(np.int64).sum()) * self.elem_words
        dev = torch.device("cuda", device)

        def view(ptr, n, typestr, dtype):
            if n == 0 or not ptr:
                return torch.zeros(0, dtype=dtype, device=dev)
            return torch.as_tensor(_DeviceArray(ptr, n, typestr), device=dev)
        return view(d, total, "<i8", torch.int64), view(st, self.n, "<i8", torch.int64), \
            view(sz, self.n, "<i4", torch.int32)

    def export(self, d_dst_ptr, stride, d_sizes_ptr):
        check(lib().sks_sketch_set_export(self.h, C.c_void_p(d_dst_ptr), stride,
                                          C.c_void_p(d_sizes_ptr)))


def build_info():
    """'src:<hash>' of the sources libsks.so was linked from (srchash.py)."""
    return lib().sks_build_info().decode()
