"""Python binding of libgol.so (include/gol.h) -- the MI355X Game of Life engine.

Thin ctypes layer used by bench.py, the tests and __graft_entry__: no compute
happens here.  Every call goes to the C ABI, whose kernels run on the GPU; there
is no CPU fallback.  Loading fails loudly (GolError) if libgol.so is missing.

The directory name is not a Python identifier, so load it with `load_package()`
from __graft_entry__.py, or importlib with an explicit path.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# GOL_LIB: dev-only override (A/B of kernel builds in tools/); the product loads libgol.so
LIB_PATH = os.environ.get("GOL_LIB") or os.path.join(HERE, "libgol.so")
CLI_PATH = os.path.join(HERE, "gol")

GOL_OK, GOL_EINVAL, GOL_ENOMEM, GOL_EHIP, GOL_ERCCL, GOL_EIO, GOL_ESTATE, GOL_EXFER = range(8)
# gol_sched_kind (include/gol.h)
OP_EXCHANGE, OP_WAIT_EXCHANGE, OP_LAUNCH, OP_BAND, OP_INTERIOR, OP_EXCHANGE_ASYNC = range(6)
OP_NAMES = ["EXCHANGE", "WAIT_EXCHANGE", "LAUNCH", "BAND", "INTERIOR", "EXCHANGE_ASYNC"]
SEM_GLOBAL, SEM_REF_STRIPES = 0, 1

# (birth, survive) masks; bit n <=> n live neighbours
REF_RULE = (0, 1 << 2)  # effective rule of Parallel_Life_MPI.cpp:44-50 ("B/S2")
CONWAY = (1 << 3, (1 << 2) | (1 << 3))  # B3/S23

# Every symbol include/gol.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "gol_config_init", "gol_create", "gol_load_ascii", "gol_store_ascii",
    "gol_load_packed", "gol_store_packed", "gol_init_random", "gol_step", "gol_sync",
    "gol_digest", "gol_destroy", "gol_last_error", "gol_set_timing", "gol_get_timing",
    "gol_reset_timing", "gol_info", "gol_rank_rows", "gol_comm_unique_id",
    "gol_create_rank", "gol_create_group", "gol_group_step", "gol_plan_info",
    "gol_create_rank_transport", "gol_round_schedule", "gol_plan_handoff",
    "gol_plan_resident", "gol_plan_skew", "gol_plan_columns", "gol_plan_tuning",
    "gol_digest_rows", "gol_comm_info", "gol_plan_model", "gol_plan_passes",
    "gol_plan_resident_rows", "gol_plan_exchange",
]

# gol_plan_tuning's variants (plan.cpp kTuneVariantNames): 0 = the models' plan
TUNE_VARIANTS = ["models", "no_half_strip", "skew_0.95", "skew_1.05", "other_block_kind"]


class GolError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"gol status {status}: {msg}")
        self.status = status


class Config(ctypes.Structure):
    _fields_ = [
        ("birth_mask", ctypes.c_uint32),
        ("survive_mask", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("semantics", ctypes.c_uint32),
        ("ref_ranks", ctypes.c_uint32),
        ("tb_depth", ctypes.c_uint32),
        ("halo_depth", ctypes.c_uint32),
        ("rows_per_wave", ctypes.c_uint32),
        ("handoff", ctypes.c_uint32),
        ("streams", ctypes.c_uint32),
        ("strip_lanes", ctypes.c_uint32),
        ("word_planes", ctypes.c_uint32),
        ("resident", ctypes.c_uint32),
        ("exchange_overlap", ctypes.c_uint32),
    ]


class Timing(ctypes.Structure):
    _fields_ = [
        ("launches", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double),
        ("cell_gens", ctypes.c_double),
        ("cell_gens_computed", ctypes.c_double),
        ("streams", ctypes.c_uint32),
        ("struct_size", ctypes.c_uint32),  # in: sizeof(gol_timing) (gol.h)
        ("launches_issued", ctypes.c_uint64),
        ("launch_rows", ctypes.c_double),
        ("exchanges", ctypes.c_uint64),
        ("exchange_ms", ctypes.c_double),
        ("rounds", ctypes.c_uint64),
        ("round_ms", ctypes.c_double),
        ("exchange_exposed_ms", ctypes.c_double),
    ]


class PlanSummary(ctypes.Structure):
    _fields_ = [
        ("tb_depth", ctypes.c_uint32), ("halo_depth", ctypes.c_uint32),
        ("plans", ctypes.c_uint32), ("distinct_plans", ctypes.c_uint32),
        ("rows_lo", ctypes.c_int64), ("rows_hi", ctypes.c_int64),
        ("rows_per_wave", ctypes.c_int64),
        ("rows_old", ctypes.c_int32), ("units_old", ctypes.c_int32),
        ("strips", ctypes.c_int32), ("lane_shift", ctypes.c_int32),
        ("total_units", ctypes.c_int64), ("half_units", ctypes.c_int64),
        ("blocks", ctypes.c_int64),
        ("handoff", ctypes.c_int32), ("tail_off", ctypes.c_int32),
        ("candidates", ctypes.c_uint32), ("passes", ctypes.c_uint32),
    ]


class SchedOp(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_uint32),
        ("depth", ctypes.c_uint32),
        ("shrink", ctypes.c_uint32),
        ("nseg", ctypes.c_uint32),
        ("out_lo", ctypes.c_int64 * 2),
        ("out_hi", ctypes.c_int64 * 2),
    ]


# gol_halo_exchange_fn(ctx, send_up, recv_up, send_down, recv_down, bytes) -> int
HALO_EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64)


class Transport(ctypes.Structure):
    _fields_ = [("exchange", HALO_EXCHANGE_FN), ("ctx", ctypes.c_void_p)]


def build(force=False):
    """Compile libgol.so and the CLI in-tree (hipcc --offload-arch=gfx950)."""
    args = ["make", "-s", "-C", HERE, "-j8"]
    if force:
        subprocess.run(["make", "-s", "-C", HERE, "clean"], check=True)
    subprocess.run(args, check=True)


_lib = None


def lib():
    """Load libgol.so (torch first, so one HIP runtime serves the process)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GolError(-1, f"{LIB_PATH} not built; run __graft_entry__.build()")
    try:  # share torch's HIP runtime when torch is present (same SONAME)
        import torch  # noqa: F401
    except Exception:
        pass
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    L.gol_config_init.argtypes = [ctypes.POINTER(Config)]
    L.gol_config_init.restype = None
    L.gol_create.argtypes = [u64, u64, ctypes.POINTER(Config), ctypes.POINTER(vp)]
    L.gol_create_rank.argtypes = [u64, u64, ctypes.POINTER(Config), i32, i32, ctypes.c_char_p,
                                  ctypes.POINTER(vp)]
    L.gol_load_ascii.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
    L.gol_store_ascii.argtypes = [vp, vp, ctypes.c_size_t]
    L.gol_load_packed.argtypes = [vp, vp, u64]
    L.gol_store_packed.argtypes = [vp, vp, u64]
    L.gol_init_random.argtypes = [vp, u64]
    L.gol_step.argtypes = [vp, u64]
    L.gol_sync.argtypes = [vp]
    L.gol_digest.argtypes = [vp, pu64, pu64]
    L.gol_destroy.argtypes = [vp]
    L.gol_destroy.restype = None
    L.gol_last_error.argtypes = []
    L.gol_last_error.restype = ctypes.c_char_p
    L.gol_set_timing.argtypes = [vp, i32]
    L.gol_get_timing.argtypes = [vp, ctypes.POINTER(Timing)]
    L.gol_reset_timing.argtypes = [vp]
    L.gol_info.argtypes = [vp, pu64, pu64, pu64, pu64, ctypes.POINTER(u32), ctypes.POINTER(u32),
                           ctypes.POINTER(u32)]
    L.gol_rank_rows.argtypes = [u64, i32, i32, pu64, pu64]
    L.gol_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.gol_create_group.argtypes = [u64, u64, ctypes.POINTER(Config), i32,
                                   ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp)]
    L.gol_group_step.argtypes = [ctypes.POINTER(vp), i32, u64]
    L.gol_plan_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
    L.gol_plan_handoff.argtypes = [vp, ctypes.POINTER(u32)]
    L.gol_plan_resident.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
    L.gol_plan_skew.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
    L.gol_plan_columns.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
    L.gol_create_rank_transport.argtypes = [u64, u64, ctypes.POINTER(Config), i32, i32,
                                            ctypes.POINTER(Transport), ctypes.POINTER(vp)]
    pf32 = ctypes.POINTER(ctypes.c_float)
    L.gol_plan_tuning.argtypes = [vp, ctypes.POINTER(u32), pf32, pf32]
    L.gol_plan_passes.argtypes = [vp, ctypes.POINTER(u32)]
    L.gol_plan_exchange.argtypes = [vp, ctypes.POINTER(u32), pf32, pf32]
    L.gol_plan_resident_rows.argtypes = [vp] + [ctypes.POINTER(u32)] * 4
    L.gol_digest_rows.argtypes = [vp, u64, u64, pu64, pu64]
    pi32 = ctypes.POINTER(ctypes.c_int)
    L.gol_comm_info.argtypes = [vp, pi32, pi32, pi32, pi32, pi32]
    L.gol_round_schedule.argtypes = [u64, u64, ctypes.POINTER(Config), i32, i32, u64, i32,
                                     ctypes.POINTER(SchedOp), u64, pu64, ctypes.POINTER(u32),
                                     ctypes.POINTER(u32)]
    L.gol_plan_model.argtypes = [u64, u64, ctypes.POINTER(Config), i32, i32, i32, i32, i32,
                                 ctypes.POINTER(PlanSummary)]
    for name in ["gol_create", "gol_create_rank", "gol_load_ascii", "gol_store_ascii",
                 "gol_load_packed", "gol_store_packed", "gol_init_random", "gol_step",
                 "gol_sync", "gol_digest", "gol_set_timing", "gol_get_timing",
                 "gol_reset_timing", "gol_info", "gol_rank_rows", "gol_comm_unique_id",
                 "gol_create_group", "gol_group_step", "gol_plan_info", "gol_plan_handoff",
                 "gol_plan_resident", "gol_plan_skew", "gol_plan_columns",
                 "gol_create_rank_transport", "gol_round_schedule", "gol_plan_tuning",
                 "gol_digest_rows", "gol_comm_info", "gol_plan_model", "gol_plan_passes",
                 "gol_plan_resident_rows", "gol_plan_exchange"]:
        getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


def _check(st):
    if st != GOL_OK:
        raise GolError(st, lib().gol_last_error().decode(errors="replace"))


def make_config(rule=REF_RULE, device=-1, semantics=SEM_GLOBAL, ref_ranks=1, tb_depth=0,
                halo_depth=0, rows_per_wave=0, handoff=0, streams=0, strip_lanes=0,
                word_planes=0, resident=0, exchange_overlap=0):
    c = Config()
    lib().gol_config_init(ctypes.byref(c))
    c.birth_mask, c.survive_mask = rule
    c.device = device
    c.semantics = semantics
    c.ref_ranks = ref_ranks
    c.tb_depth = tb_depth
    c.halo_depth = halo_depth
    c.rows_per_wave = rows_per_wave
    c.handoff = handoff
    c.streams = streams
    c.strip_lanes = strip_lanes
    c.word_planes = word_planes
    c.resident = resident
    c.exchange_overlap = exchange_overlap
    return c


def rank_rows(h, nranks, rank):
    r0, n = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().gol_rank_rows(h, nranks, rank, ctypes.byref(r0), ctypes.byref(n)))
    return r0.value, n.value


def round_schedule(h, w, rank, nranks, gens, halo_fresh=False, **cfg_kw):
    """The launch/exchange schedule gol_step runs on stripe `rank` of `nranks`
    (gol_round_schedule; host-only).  Returns (ops, K, Hx), ops as dicts with
    kind (OP_*), depth, shrink and segs [(out_lo, out_hi), ...] in local rows."""
    cfg = make_config(**cfg_kw)
    n, K, Hx = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().gol_round_schedule(h, w, ctypes.byref(cfg), rank, nranks, gens,
                                    1 if halo_fresh else 0, None, 0, ctypes.byref(n),
                                    ctypes.byref(K), ctypes.byref(Hx)))
    arr = (SchedOp * max(1, n.value))()
    _check(lib().gol_round_schedule(h, w, ctypes.byref(cfg), rank, nranks, gens,
                                    1 if halo_fresh else 0, arr, n.value, ctypes.byref(n),
                                    ctypes.byref(K), ctypes.byref(Hx)))
    ops = [{"kind": o.kind, "depth": o.depth, "shrink": o.shrink,
            "segs": [(o.out_lo[i], o.out_hi[i]) for i in range(o.nseg)]}
           for o in arr[:n.value]]
    return ops, K.value, Hx.value


def plan_model(h, w, rank=0, nranks=1, cus=256, occ_classic=2, occ_hand=2, **cfg_kw):
    """gol_plan_model (host only, no GPU): the first full-depth launch plan the
    engine would build on a device of `cus` CUs with those occupancies (256-thread
    workgroups per CU), before the autotuner.  Returns a dict of PlanSummary."""
    cfg = make_config(**cfg_kw)
    out = PlanSummary()
    _check(lib().gol_plan_model(h, w, ctypes.byref(cfg), rank, nranks, cus, occ_classic,
                                occ_hand, ctypes.byref(out)))
    return {k: getattr(out, k) for k, _ in PlanSummary._fields_ if k != "reserved"}


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(lib().gol_comm_unique_id(buf))
    return buf.raw


class Engine:
    """One field (or one rank's stripe of it) resident on one GPU."""

    def __init__(self, h, w, rule=REF_RULE, device=-1, semantics=SEM_GLOBAL, ref_ranks=1,
                 tb_depth=0, halo_depth=0, rows_per_wave=0, rank=None, nranks=1, uid=None,
                 handoff=0, streams=0, strip_lanes=0, word_planes=0, transport=None,
                 resident=0, exchange_overlap=0, _handle=None):
        """transport: for a rank engine, a callable (send_up, send_down) -> (recv_up,
        recv_down) of bytes objects (None where there is no neighbour) used instead
        of RCCL (gol_create_rank_transport)."""
        self.h, self.w = h, w
        self.wq = (w + 63) // 64
        self._tp = None
        cfg = make_config(rule, device, semantics, ref_ranks, tb_depth, halo_depth,
                          rows_per_wave, handoff, streams, strip_lanes, word_planes, resident,
                          exchange_overlap)
        handle = ctypes.c_void_p()
        if _handle is not None:
            handle = _handle
        elif rank is None:
            _check(lib().gol_create(h, w, ctypes.byref(cfg), ctypes.byref(handle)))
        elif transport is not None:
            self._tp = _make_transport(transport)
            _check(lib().gol_create_rank_transport(h, w, ctypes.byref(cfg), rank, nranks,
                                                   ctypes.byref(self._tp[0]),
                                                   ctypes.byref(handle)))
        else:
            if uid is None or len(uid) != 128:
                raise GolError(GOL_EINVAL, "rank engines need a 128-byte RCCL unique id")
            _check(lib().gol_create_rank(h, w, ctypes.byref(cfg), rank, nranks, uid,
                                         ctypes.byref(handle)))
        self._h = handle
        h_, w_, r0, rows = (ctypes.c_uint64() for _ in range(4))
        k, hx, rpw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().gol_info(self._h, ctypes.byref(h_), ctypes.byref(w_), ctypes.byref(r0),
                              ctypes.byref(rows), ctypes.byref(k), ctypes.byref(hx),
                              ctypes.byref(rpw)))
        self.row0, self.rows, self.tb_depth, self.halo_depth = r0.value, rows.value, k.value, hx.value
        self.rows_per_wave = rpw.value
        sl, rp, wp = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().gol_plan_info(self._h, ctypes.byref(sl), ctypes.byref(rp), ctypes.byref(wp)))
        self.strip_lanes = sl.value
        self.word_planes = wp.value
        ho = ctypes.c_uint32()
        _check(lib().gol_plan_handoff(self._h, ctypes.byref(ho)))
        self.handoff = bool(ho.value)
        on, nb, ns = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().gol_plan_resident(self._h, ctypes.byref(on), ctypes.byref(nb), ctypes.byref(ns)))
        # resident kernel: (bands, strips) of its tiles, or None
        self.resident = (nb.value, ns.value) if on.value else None
        rr = [ctypes.c_uint32() for _ in range(4)]
        _check(lib().gol_plan_resident_rows(self._h, *(ctypes.byref(v) for v in rr)))
        # resident kernel: rows per wavefront, band rows, epoch K, generations
        # between the wavefronts' LDS row swaps (1: every one), or None
        self.resident_rows = tuple(v.value for v in rr) if on.value else None
        ro, ry, uo = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().gol_plan_skew(self._h, ctypes.byref(ro), ctypes.byref(ry), ctypes.byref(uo)))
        # age-skewed row blocks: (rows_old, rows_young, units_old), or None
        self.age_skew = (ro.value, ry.value, uo.value) if ro.value else None
        st, hu, hg = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().gol_plan_columns(self._h, ctypes.byref(st), ctypes.byref(hu), ctypes.byref(hg)))
        # (strips per row block, half-strip units, half-strip lane groups)
        self.columns = (st.value, hu.value, hg.value)
        tv, tu, mu = ctypes.c_uint32(), ctypes.c_float(), ctypes.c_float()
        _check(lib().gol_plan_tuning(self._h, ctypes.byref(tv), ctypes.byref(tu), ctypes.byref(mu)))
        # autotuner outcome of the first full-depth plan: (variant name, best launch us
        # of the plan that runs, of the models' plan); us 0 = not timed
        self.tuning = (TUNE_VARIANTS[tv.value] if tv.value < len(TUNE_VARIANTS) else str(tv.value),
                       round(tu.value, 2), round(mu.value, 2))
        np_ = ctypes.c_uint32()
        _check(lib().gol_plan_passes(self._h, ctypes.byref(np_)))
        self.passes = np_.value  # passes per full-depth launch (multi-pass launches)
        xm, xb, xo = ctypes.c_uint32(), ctypes.c_float(), ctypes.c_float()
        _check(lib().gol_plan_exchange(self._h, ctypes.byref(xm), ctypes.byref(xb), ctypes.byref(xo)))
        # exchange mode of a stripe engine ("blocking" / "overlapped", None without
        # exchanges) and, when it was chosen by timing at create (exchange_overlap =
        # 0 over RCCL), the max over ranks of each mode's best ms per round
        self.exchange = ({1: "blocking", 2: "overlapped"}.get(xm.value),
                         round(xb.value, 4), round(xo.value, 4))

    def close(self):
        if self._h:
            lib().gol_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load_ascii(self, data: bytes):
        _check(lib().gol_load_ascii(self._h, data, len(data)))

    def store_ascii(self, nbytes=None) -> bytes:
        n = nbytes if nbytes is not None else self.rows * (self.w + 1)
        buf = ctypes.create_string_buffer(n)
        _check(lib().gol_store_ascii(self._h, buf, n))
        return buf.raw

    def load_packed(self, arr):
        import numpy as np
        a = np.ascontiguousarray(arr, dtype=np.uint64)
        _check(lib().gol_load_packed(self._h, a.ctypes.data, a.shape[1]))

    def store_packed(self, rows=None):
        import numpy as np
        rows = rows if rows is not None else self.rows
        a = np.zeros((rows, self.wq), dtype=np.uint64)
        _check(lib().gol_store_packed(self._h, a.ctypes.data, self.wq))
        return a

    def init_random(self, seed=1):
        _check(lib().gol_init_random(self._h, seed))

    def step(self, gens):
        _check(lib().gol_step(self._h, gens))

    def sync(self):
        _check(lib().gol_sync(self._h))

    def digest(self):
        live, hsh = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().gol_digest(self._h, ctypes.byref(live), ctypes.byref(hsh)))
        return live.value, hsh.value

    def digest_rows(self, row0, rows):
        """gol_digest over field rows [row0, row0 + rows) only."""
        live, hsh = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().gol_digest_rows(self._h, row0, rows, ctypes.byref(live), ctypes.byref(hsh)))
        return live.value, hsh.value

    def comm_info(self):
        """RCCL communicator of a rank engine: dict(count, rank, peer_up, peer_down,
        device) as RCCL reports them (gol_comm_info)."""
        v = [ctypes.c_int() for _ in range(5)]
        _check(lib().gol_comm_info(self._h, *(ctypes.byref(x) for x in v)))
        return dict(zip(("count", "rank", "peer_up", "peer_down", "device"), (x.value for x in v)))

    def set_timing(self, every=1):
        """Time every `every`-th stencil launch with HIP events (0/False = off)."""
        _check(lib().gol_set_timing(self._h, int(every)))

    def reset_timing(self):
        _check(lib().gol_reset_timing(self._h))

    def timing(self):
        t = Timing(struct_size=ctypes.sizeof(Timing))
        _check(lib().gol_get_timing(self._h, ctypes.byref(t)))
        if t.struct_size != ctypes.sizeof(Timing):
            raise GolError(GOL_ESTATE, f"libgol.so's gol_timing is {t.struct_size} bytes, "
                                       f"this binding's {ctypes.sizeof(Timing)}")
        return {k: getattr(t, k) for k, _ in Timing._fields_ if k != "struct_size"}


def _make_transport(fn):
    """Wrap a Python halo exchange `fn(send_up, send_down) -> (recv_up, recv_down)`
    (bytes or None) as a gol_transport; keep the result alive with the engine."""
    def cb(ctx, send_up, recv_up, send_dn, recv_dn, nbytes):
        try:
            su = ctypes.string_at(send_up, nbytes) if send_up else None
            sd = ctypes.string_at(send_dn, nbytes) if send_dn else None
            ru, rd = fn(su, sd)
            for ptr, data in ((recv_up, ru), (recv_dn, rd)):
                if ptr:
                    if data is None or len(data) != nbytes:
                        return 2
                    ctypes.memmove(ptr, data, nbytes)
            return 0
        except Exception:  # a Python error must not unwind through C
            import traceback
            traceback.print_exc()
            return 1
    cfn = HALO_EXCHANGE_FN(cb)
    return Transport(cfn, None), cfn


class Group:
    """`nranks` stripe engines of one field in this process (gol_create_group):
    the multi-GPU partition/halo logic with device-copy transport; stripes may
    share a GPU."""

    def __init__(self, h, w, nranks, devices=None, rule=REF_RULE, tb_depth=0, halo_depth=0,
                 rows_per_wave=0, handoff=0, strip_lanes=0, word_planes=0, exchange_overlap=0):
        self.h, self.w, self.n = h, w, nranks
        cfg = make_config(rule, -1 if devices else 0, SEM_GLOBAL, 1, tb_depth, halo_depth,
                          rows_per_wave, handoff, strip_lanes=strip_lanes,
                          word_planes=word_planes, exchange_overlap=exchange_overlap)
        hs = (ctypes.c_void_p * nranks)()
        devs = (ctypes.c_int * nranks)(*(devices or [0] * nranks))
        _check(lib().gol_create_group(h, w, ctypes.byref(cfg), nranks, devs, hs))
        self._hs = hs
        self.members = [Engine(h, w, _handle=ctypes.c_void_p(hs[r])) for r in range(nranks)]

    def close(self):
        for m in self.members:
            m.close()
        self.members = []

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def step(self, gens):
        _check(lib().gol_group_step(self._hs, self.n, gens))

    def sync(self):
        for m in self.members:
            m.sync()

    def init_random(self, seed=1):
        for m in self.members:
            m.init_random(seed)

    def load_packed(self, arr):
        for m in self.members:
            m.load_packed(arr[m.row0:m.row0 + m.rows])

    def load_ascii(self, data: bytes):
        for m in self.members:
            m.load_ascii(data[m.row0 * (self.w + 1):(m.row0 + m.rows) * (self.w + 1)])

    def store_packed(self):
        import numpy as np
        return np.concatenate([m.store_packed() for m in self.members])

    def store_ascii(self) -> bytes:
        return b"".join(m.store_ascii() for m in self.members)

    def digest(self):
        live = hsh = 0
        for m in self.members:
            a, b = m.digest()
            live += a
            hsh = (hsh + b) & 0xFFFFFFFFFFFFFFFF
        return live, hsh
