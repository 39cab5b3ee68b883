"""ctypes wrapper for the CPU oracle (liboracle.so, built from gol_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / the timed CPU port.  The product
(libgol.so, the `gol` CLI) never loads it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GOL_ORACLE_LIB: another build of gol_oracle.c (tools/asan_cpu_suite.sh: the sanitizer build)
_LIB = os.environ.get("GOL_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")

# Rule masks: bit n set <=> a cell with n live neighbours is born / survives.
REF_RULE = (0, 1 << 2)  # the reference's effective rule "B/S2" (Parallel_Life_MPI.cpp:44-50)
CONWAY = (1 << 3, (1 << 2) | (1 << 3))  # B3/S23
HIGHLIFE = ((1 << 3) | (1 << 6), (1 << 2) | (1 << 3))  # B36/S23


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _lib():
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(
        os.path.join(_HERE, "gol_oracle.c")
    ):
        build()
    lib = ctypes.CDLL(_LIB)
    i64, u64, u32, i32 = ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    vp = ctypes.c_void_p
    lib.oracle_ref_program.argtypes = [vp, ctypes.c_size_t, i32, i32, i32, i32, u32, u32, vp, i32]
    lib.oracle_ref_program.restype = i32
    lib.oracle_ref_stripe.argtypes = [i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    lib.oracle_ref_stripe.restype = i32
    lib.oracle_ref_baseline.argtypes = [i32, i32, i32, i32, u64, u32, u32]
    lib.oracle_ref_baseline.restype = i64
    lib.oracle_bp_init_random.argtypes = [vp, i64, i64, i64, u64]
    lib.oracle_bp_init_random_rows.argtypes = [vp, i64, i64, i64, i64, u64]
    lib.oracle_bp_digest.argtypes = [vp, i64, i64, i64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.oracle_bp_pack_ascii.argtypes = [vp, ctypes.c_size_t, i64, i64, vp, i64]
    lib.oracle_bp_pack_ascii.restype = i32
    lib.oracle_bp_unpack_ascii.argtypes = [vp, i64, i64, i64, vp]
    lib.oracle_bp_step.argtypes = [vp, vp, i64, i64, i64, u32, u32, i32]
    lib.oracle_bp_run.argtypes = [vp, i64, i64, i64, i64, u32, u32, i32]
    lib.oracle_bp_run.restype = i32
    return lib


_L = None


def lib():
    global _L
    if _L is None:
        _L = _lib()
    return _L


def words(w):
    return (w + 63) // 64


def ref_program(data: bytes, h: int, w: int, epochs: int, P: int = 1, rule=REF_RULE,
                parallel: bool = True) -> bytes:
    """Bytes the reference writes to output.txt under `mpirun -np P`."""
    out = ctypes.create_string_buffer(h * (w + 1))
    buf = ctypes.create_string_buffer(data, len(data))
    rc = lib().oracle_ref_program(buf, len(data), h, w, epochs, P, rule[0], rule[1], out,
                                  1 if parallel else 0)
    if rc != 0:
        raise ValueError(f"oracle_ref_program failed rc={rc}")
    return out.raw


def ref_stripe(h, P, r):
    s, n = ctypes.c_int(), ctypes.c_int()
    if lib().oracle_ref_stripe(h, P, r, ctypes.byref(s), ctypes.byref(n)) != 0:
        raise ValueError("bad stripe")
    return s.value, n.value


def ref_baseline(rows_per_thread, w, gens, threads, seed=1, rule=REF_RULE):
    return lib().oracle_ref_baseline(rows_per_thread, w, gens, threads, seed, rule[0], rule[1])


def bp_random(h, w, seed=1, stride=None):
    stride = stride or words(w)
    g = np.zeros((h, stride), dtype=np.uint64)
    lib().oracle_bp_init_random(g.ctypes.data, h, w, stride, seed)
    return g


def bp_random_rows(row0, h, w, seed=1):
    """Rows [row0, row0 + h) of bp_random(row0 + h, w, seed), without the rest."""
    g = np.zeros((h, words(w)), dtype=np.uint64)
    lib().oracle_bp_init_random_rows(g.ctypes.data, row0, h, w, words(w), seed)
    return g


def bp_digest(g, w):
    h, stride = g.shape
    live, hsh = ctypes.c_uint64(), ctypes.c_uint64()
    g = np.ascontiguousarray(g)
    lib().oracle_bp_digest(g.ctypes.data, h, w, stride, ctypes.byref(live), ctypes.byref(hsh))
    return live.value, hsh.value


def bp_pack(data: bytes, h, w, stride=None):
    stride = stride or words(w)
    g = np.zeros((h, stride), dtype=np.uint64)
    if lib().oracle_bp_pack_ascii(data, len(data), h, w, g.ctypes.data, stride) != 0:
        raise ValueError("bad ascii length")
    return g


def bp_unpack(g, w) -> bytes:
    h, stride = g.shape
    g = np.ascontiguousarray(g)
    out = ctypes.create_string_buffer(h * (w + 1))
    lib().oracle_bp_unpack_ascii(g.ctypes.data, h, w, stride, out)
    return out.raw


def bp_run(g, w, gens, rule=REF_RULE, threads=8):
    """Evolve a packed field `gens` generations (dead boundary); returns a new array."""
    g = np.ascontiguousarray(g).copy()
    h, stride = g.shape
    if lib().oracle_bp_run(g.ctypes.data, h, w, stride, gens, rule[0], rule[1], threads) != 0:
        raise MemoryError
    return g


def bp_ref_stripes(g, w, gens, P, rule=REF_RULE, threads=8):
    """REF_STRIPES:P semantics on a packed field: each rank's extended stripe
    (Parallel_Life_MPI.cpp:70-81) evolves alone with a dead boundary, the output
    keeps each rank's own rows (:149-164)."""
    h = g.shape[0]
    out = np.zeros_like(g)
    c = h // P
    for r in range(P):
        s, n = ref_stripe(h, P, r)
        sub = bp_run(g[s:s + n], w, gens, rule, threads)
        lo = r * c
        hi = h if r == P - 1 else (r + 1) * c
        out[lo:hi] = sub[lo - s:hi - s]
    return out
