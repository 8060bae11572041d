"""Session windows (BASELINE config 5): native store / GPU operator vs the exact host
WindowOperator with EventTimeSessionWindows (Flink MergingWindowSet semantics).

Oracle: the DataStream API on the host path (native off), punctuated watermark max_ts - bound
after every element. Engine: KeyedSessionOperator fed one element per micro-batch (then outputs
must be identical, late handling included) or in larger batches without late data (then the
sessions formed are identical because session merging is associative).
"""
from collections import Counter

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.api.time import Time, TimeCharacteristic
from mxstream.api.watermarks import AssignerWithPunctuatedWatermarks, Watermark
from mxstream.api.windowing import EventTimeSessionWindows
from mxstream.ops import expr as E
from mxstream.ops import kernels as K
from mxstream.runtime.session_operator import KeyedSessionOperator

LONG_MIN = -(1 << 63)


class _Punct(AssignerWithPunctuatedWatermarks):
    periodic = False

    def __init__(self, bound):
        self.bound = bound
        self.max = LONG_MIN

    def extract_timestamp(self, e, prev):
        self.max = max(self.max, e[1])
        return e[1]

    def check_and_get_next_watermark(self, last, ts):
        return Watermark(self.max - self.bound)


def oracle(events, gap, bound, lateness):
    out = []
    env = StreamExecutionEnvironment(1)
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    env.config.native = "off"
    (env.from_collection([(k, t, v, 1) for k, t, v in events])
     .assign_timestamps_and_watermarks(_Punct(bound))
     .key_by(lambda e: e[0])
     .window(EventTimeSessionWindows.with_gap(Time.milliseconds(gap)))
     .allowed_lateness(Time.milliseconds(lateness))
     .reduce(lambda a, b: (a[0], a[1], a[2] + b[2], a[3] + b[3]),
             lambda key, w, els, col: [col.collect((key, w.start, w.end, e[2], e[3])) for e in els])
     .collect(out))
    env.execute("session-oracle")
    return Counter(out)


def engine(events, gap, bound, lateness, device="cpu", batch=1, **kw):
    op = KeyedSessionOperator(gap=gap, lateness=lateness, agg=K.AGG_SUM_I64, device=device,
                              max_keys=1 << 10, batch_capacity=max(batch, 64), ooo_bound=bound,
                              **kw)
    out = Counter()

    def take(rows):
        for k, s, e, r, c in zip(rows.keys, rows.start, rows.end, rows.raw, rows.counts):
            out[(int(k), int(s), int(e), int(r), int(c))] += 1

    for i in range(0, len(events), batch):
        chunk = events[i:i + batch]
        k = torch.tensor([e[0] for e in chunk], dtype=torch.int64, device=device)
        t = torch.tensor([e[1] for e in chunk], dtype=torch.int64, device=device)
        v = torch.tensor([e[2] for e in chunk], dtype=torch.int64, device=device)
        take(op.process(k, t, v))
    take(op.finish())
    return out, op


events_st = st.lists(st.tuples(st.integers(0, 5), st.integers(0, 5_000), st.integers(0, 100)),
                     min_size=1, max_size=50)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=events_st, gap=st.sampled_from([1, 50, 300, 1000]),
       bound=st.sampled_from([0, 200, 2000]), lateness=st.sampled_from([0, 500]))
def test_store_equals_flink_per_element(events, gap, bound, lateness):
    got, _ = engine(events, gap, bound, lateness)
    assert got == oracle(events, gap, bound, lateness)


@settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 10_000), gap=st.sampled_from([10, 100, 400]),
       batch=st.sampled_from([7, 64, 500]))
def test_store_batched_no_late_data(seed, gap, batch):
    rng = np.random.default_rng(seed)
    n = 600
    ts = np.sort(rng.integers(0, 20_000, n))
    ts = ts + rng.integers(-50, 50, n)  # disorder < bound: nothing is late
    events = [(int(k), int(t), int(v)) for k, t, v in
              zip(rng.integers(0, 20, n), ts, rng.integers(0, 100, n))]
    got, op = engine(events, gap, 100, 0, batch=batch)
    assert op.metrics.num_late_records_dropped == 0
    assert got == oracle(events, gap, 100, 0)


def test_session_late_refire_and_drop():
    # gap 10: a=[0,10) fires at wm>=9; a late element inside lateness re-fires the merged session;
    # an element past cleanup is dropped.
    ev = [(1, 0, 5), (1, 3, 1), (1, 40, 2), (1, 5, 10), (1, 100, 1), (1, 2, 7)]
    got, op = engine(ev, 10, 0, 40)
    assert got == oracle(ev, 10, 0, 40)
    assert op.metrics.num_late_records_dropped == 1


def test_session_map_filter_epilogue():
    op = KeyedSessionOperator(gap=100, agg=K.AGG_SUM_I64, max_keys=64, batch_capacity=64,
                              map_prog=E.compile_expr(E.var(E.VAR_RESULT) * 2.0),
                              filter_prog=E.compile_expr(E.var(E.VAR_COUNT) >= 2))
    k = torch.tensor([1, 1, 2, 3, 3, 3])
    t = torch.tensor([0, 50, 10, 0, 90, 180])
    v = torch.tensor([1, 2, 5, 1, 1, 1])
    got = []
    for rows in (op.process(k, t, v), op.finish()):
        got += zip(rows.keys.tolist(), rows.values.tolist(), rows.counts.tolist())
    got.sort()
    assert got == [(1, 6.0, 2), (3, 6.0, 3)]


def test_spill_set_builder():
    from mxstream.ops.native import load

    s = load().SessionStore(10, 0, K.AGG_SUM_I64)
    s.process(np.array([5, 9, 12], np.int64), np.array([0, 0, 0], np.int64),
              np.array([1, 1, 1], np.int64), LONG_MIN)
    arr = s.spill_set(4)
    assert sorted(int(x) for x in arr if x != -1) == [5, 9, 12]


def test_store_cold_tier_promotion_equals_hot():
    """Sessions inserted as cold rows (spilled, fired, waiting for cleanup) behave exactly like
    hot ones: late records promote them (or find them cleaned), cleanup releases the keys."""
    from mxstream.ops.native import load

    m = load()
    rng = np.random.default_rng(7)
    hot = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    cold = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    n = 400
    keys = rng.integers(0, 300, n)
    starts = rng.integers(0, 5000, n)
    rows = [np.unique(keys)]
    k = rows[0].astype(np.int64)
    s = (k * 17) % 5000
    e = s + 100
    acc = k * 3
    cnt = np.ones_like(k)
    flags = np.ones_like(k)
    hot.insert(k, s, e, acc, cnt, flags, False)
    cold.insert(k, s, e, acc, cnt, flags, True)
    assert cold.num_cold_rows() == len(k)
    outs = []
    for st_ in (hot, cold):
        d0 = st_.fire(3000, [], [], [], [])  # the operator fires every step before new data
        late = st_.process(keys.astype(np.int64), starts.astype(np.int64), np.ones(n, np.int64),
                           3000)
        fired, released = [], set(d0["released"].tolist())
        for w in (3500, 5000, 7000, (1 << 63) - 1):
            d = st_.fire(w, [], [], [], [])
            fired.append(sorted(zip(d["keys"].tolist(), d["start"].tolist(), d["raw"].tolist())))
            released |= set(d["released"].tolist())
        outs.append((late, fired, released))
    assert outs[0] == outs[1]
    assert outs[0][2] == set(k.tolist()) | set(keys.tolist())
    assert cold.num_keys() == 0 and hot.num_keys() == 0


@pytest.mark.parametrize("spread", ["dense", "sparse"])
def test_store_cold_index_lookup_equals_hot(spread):
    """Few revisited keys in a large cold chunk take the chunk's sorted row index (radix-sorted
    for keys within 2^32 of each other, a comparison sort otherwise): same results as a store
    that holds the same sessions hot."""
    from mxstream.ops.native import load

    m = load()
    rng = np.random.default_rng(11)
    nk = 20_000
    if spread == "dense":
        k = np.arange(5_000_000, 5_000_000 + nk, dtype=np.int64)
    else:
        k = np.unique(rng.integers(-(1 << 62), 1 << 62, nk)).astype(np.int64)
    rng.shuffle(k)  # eviction order is slot order, not key order
    s = (np.abs(k) % 4000).astype(np.int64)
    e = s + 100
    ones = np.ones_like(k)
    hot = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    cold = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    hot.insert(k, s, e, k % 97, ones, ones, False)
    cold.insert(k, s, e, k % 97, ones, ones, True)
    pick = rng.choice(k, 300, replace=False)
    ts = (np.abs(pick) % 4000) + 50  # inside the stored session: merges into it
    outs = []
    for st_ in (hot, cold):
        st_.fire(3000, [], [], [], [])
        late = st_.process(pick.astype(np.int64), ts.astype(np.int64), np.full(300, 5, np.int64),
                           3000)
        d = st_.fire((1 << 63) - 1, [], [], [], [])
        outs.append((late, sorted(zip(d["keys"].tolist(), d["start"].tolist(),
                                      d["raw"].tolist(), d["counts"].tolist()))))
    assert outs[0] == outs[1]
    assert cold.num_keys() == 0


def test_store_extract_parallel_chunk_scan():
    """extract_packed over several large cold chunks of scattered dense keys (the promote path
    of config 5 with revisits): the chunks are scanned in parallel; the packed slot records
    equal the inserted sessions of the wanted keys, in key order, and the rows leave the store."""
    from mxstream.ops.native import load

    m = load()
    rng = np.random.default_rng(5)
    st_ = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    nk, nchunks = 600_000, 4
    keys = rng.permutation(nk).astype(np.int64)
    s = (keys % 4000).astype(np.int64) + 10_000
    e = s + 100
    acc = keys * 3
    ones = np.ones_like(keys)
    for c in np.array_split(np.arange(nk), nchunks):  # one cold chunk per eviction batch
        st_.insert(keys[c], s[c], e[c], acc[c], ones[c], ones[c], True)
    assert st_.num_cold_rows() == nk
    want = rng.choice(nk, 20_000, replace=False).astype(np.int64)
    ex = st_.extract_packed(want, 0, 4, 100)
    uk = np.sort(want)
    assert np.array_equal(ex["key"], uk)
    assert np.array_equal(np.sort(ex["moved"]), uk)
    rec = ex["rec"].reshape(uk.size, 4, 4)
    assert np.array_equal(rec[:, 0, 0], (uk % 4000) + 10_000)
    assert np.array_equal(rec[:, 0, 1], (uk % 4000) + 10_100)
    assert np.array_equal(rec[:, 0, 2], uk * 3)
    assert np.array_equal(rec[:, 0, 3], np.full(uk.size, 1 | (1 << 32)))
    assert not rec[:, 1:].any()
    assert np.array_equal(ex["last"], (uk % 4000) + 10_000)
    assert st_.num_cold_rows() == nk - uk.size
    again = st_.extract_packed(want, 0, 4, 100)  # already gone
    assert again["key"].size == 0


def _dense_store(m, nk, nchunks, seed):
    rng = np.random.default_rng(seed)
    st_ = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    keys = rng.permutation(nk).astype(np.int64)
    s = (keys % 4000).astype(np.int64) + 10_000
    ones = np.ones_like(keys)
    for c in np.array_split(np.arange(nk), nchunks):
        st_.insert(keys[c], s[c], s[c] + 100, keys[c] * 3, ones[c], ones[c], True)
    return st_, rng


def _rows_by_key(rows, nk):
    out, lasts = {}, {}
    for r in rows[:nk]:
        key, s, e, a, cf, last, pos, ns = (int(x) for x in r)
        assert 0 <= pos < ns <= 4
        out.setdefault(key, [None] * ns)[pos] = (s, e, a, cf)
        lasts[key] = last
    return {k: v + [("last", lasts[k])] for k, v in out.items()}


def _packed_by_key(ex):
    out = {}
    rec = ex["rec"].reshape(-1, 4, 4)
    for i, key in enumerate(ex["key"].tolist()):
        ss = [tuple(int(x) for x in rec[i, j]) for j in range(4) if rec[i, j, 3] & 0xFFFFFFFF]
        out[key] = ss + [("last", int(ex["last"][i]))]
    return out


def _extract_both(a, b, want, wm):
    rows = np.zeros((want.size * 4, 8), np.int64)
    moved = np.zeros(want.size, np.int64)
    nk, nm, nu = a.extract_rows_into(want, wm, 4, 100, rows.ctypes.data, rows.shape[0],
                                     moved.ctypes.data, moved.size)
    assert nu == np.unique(want).size
    ex = b.extract_packed(want, wm, 4, 100)
    assert _rows_by_key(rows, nk) == _packed_by_key(ex)
    assert np.array_equal(np.sort(moved[:nm]), np.sort(ex["moved"]))
    return nk, nm


def test_store_extract_rows_into_equals_extract_packed():
    """The promote path's extract into caller memory (SessionStore.extract_rows_into: the dense
    cold-row index, one lookup per wanted key) hands back exactly extract_packed's sessions:
    same keys, same slot records, same last activity, same moved keys; rows past cleanup at wm
    are dropped and the rows leave the store (a second extract finds nothing)."""
    from mxstream.ops.native import load

    m = load()
    a, rng = _dense_store(m, 300_000, 3, 11)
    b, _ = _dense_store(m, 300_000, 3, 11)
    want = np.sort(rng.choice(300_000, 40_000, replace=False)).astype(np.int64)
    wm = 10_000 + 2000 + 100 + 1000  # keys with start < 12_000 - 1 are past cleanup
    nk, nm = _extract_both(a, b, want, wm)
    assert 0 < nk < want.size and nm == want.size
    # independent of the store: the sessions inserted by _dense_store, cleanup = end - 1 + 1000
    start = want % 4000 + 10_000
    assert nk == int(np.count_nonzero(start + 100 - 1 + 1000 > wm))
    assert a.num_cold_rows() == b.num_cold_rows() == 300_000 - want.size
    nk2, _ = _extract_both(a, b, want, wm)
    assert nk2 == 0


def test_store_extract_rows_into_multi_and_hot_keys():
    """Keys with two cold rows (the index marks them and the scan takes over), keys with hot
    sessions, unsorted wanted keys and keys the store never held: still extract_packed's
    result, with several sessions of a key at positions 0, 1, ... and keys above max_sess
    staying in the store."""
    from mxstream.ops.native import load

    m = load()
    stores = []
    for _ in range(2):
        st_, _ = _dense_store(m, 50_000, 2, 3)
        k = np.array([7, 8], np.int64)
        one = np.ones(2, np.int64)
        st_.insert(k, np.array([50_000, 60_000], np.int64), np.array([50_100, 60_100], np.int64),
                   k, one, one, True)  # keys 7 and 8: a second cold row
        st_.process(np.array([20, 20, 21], np.int64), np.array([90_000, 95_000, 5], np.int64),
                    np.array([1, 2, 3], np.int64), 0)  # hot sessions of keys 20 and 21
        for t in range(5):  # key 30: five sessions, more than a slot holds
            st_.process(np.array([30], np.int64), np.array([200_000 + t * 1000], np.int64),
                        np.array([1], np.int64), 0)
        stores.append(st_)
    want = np.array([21, 8, 7, 20, 30, 999_999, 3, 4, 5, 7, 21], np.int64)  # unsorted, repeats
    nk, nm = _extract_both(stores[0], stores[1], want, 0)
    assert nm == np.unique(want).size - 1  # key 30 stays
    assert stores[0].num_keys() == stores[1].num_keys()
    # the multi keys' entries are cleared: the next extract takes the indexed path again
    w2 = np.arange(100, 200, dtype=np.int64)
    _extract_both(stores[0], stores[1], w2, 0)


def test_store_index_duplicate_keys_in_one_chunk():
    """The cold-row index of a large chunk is built by parallel row blocks: a key whose rows sit
    in two blocks of one chunk (not adjacent) must end as a multi-place key (the extract scans
    and returns both sessions); an adjacent run is one entry; keys re-evicted while an older
    row lives are multi too."""
    from mxstream.ops.native import load

    st = load().SessionStore(100, 10**9, K.AGG_SUM_I64)
    n = 200_000
    keys = np.arange(1000, 1000 + n, dtype=np.int64)
    keys[150_000] = 5  # key 5: rows 10 and 150_000 (different row blocks)
    keys[10] = 5
    keys[20], keys[21] = 6, 6  # key 6: an adjacent run
    start = np.arange(n, dtype=np.int64) * 1000
    one = np.ones(n, np.int64)
    st.insert(keys, start, start + 100, keys, one, one, True)
    ex = st.extract(np.array([5, 6, 1030], np.int64), 0, 4)
    got = sorted(zip(ex["key"].tolist(), ex["start"].tolist()))
    assert got == [(5, 10_000), (5, 150_000_000), (6, 20_000), (6, 21_000), (1030, 30_000)]
    assert st.index_stats()["multi_aborts"] >= 1
    # an older live row + a new chunk's row of the same key: multi
    k = np.array([2000, 2001], np.int64)
    st.insert(k, np.array([5, 6], np.int64) * 10**7, np.array([5, 6], np.int64) * 10**7 + 100, k,
              np.ones(2, np.int64), np.ones(2, np.int64), True)
    ex = st.extract(np.array([2000], np.int64), 0, 4)
    assert sorted(ex["start"].tolist()) == [1000 * 1000, 5 * 10**7]


@pytest.mark.parametrize("shards", [2, 8])
def test_sharded_store_equals_one_store(shards):
    """Key shards worked by the pool (csrc/session_shards.h) give the single store's results:
    element folds, evicted-row inserts (hot and cold), extracts, firings and snapshots."""
    from collections import Counter as Ctr

    from mxstream.ops.native import load

    m = load()
    rng = np.random.default_rng(17)
    a = m.SessionStore(100, 500, K.AGG_SUM_I64)
    b = m.SessionStore(100, 500, K.AGG_SUM_I64, shards)
    assert b.shards == shards
    res = {0: [], 1: []}
    for step in range(12):
        n = 3000
        k = rng.integers(0, 5000, n).astype(np.int64)
        t = (step * 400 + rng.integers(0, 600, n)).astype(np.int64)
        v = rng.integers(0, 50, n).astype(np.int64)
        ek = np.unique(rng.integers(5000, 9000, 400)).astype(np.int64)
        es = (step * 400 + (ek % 300)).astype(np.int64)
        ones = np.ones_like(ek)
        for j, st_ in enumerate((a, b)):
            r = res[j]
            r.append(st_.process(k, t, v, step * 400 - 200))
            st_.insert(ek, es, es + 100, ek % 7, ones, ones, step % 2 == 0)
            ex = st_.extract(np.unique(k[:50]), step * 400 - 200, 4)
            r.append((ex["key"].tolist(), ex["start"].tolist(), ex["acc"].tolist(),
                      sorted(ex["moved"].tolist())))
            d = st_.fire(step * 400, [], [], [], [])
            r.append((Ctr(zip(d["keys"].tolist(), d["start"].tolist(), d["raw"].tolist())),
                      sorted(d["released"].tolist())))
            r.append((st_.num_keys(), st_.num_sessions(), st_.num_cold_rows(),
                      sorted(st_.key_list().tolist())))
            sn = st_.snapshot()
            r.append(sorted(zip(sn["key"].tolist(), sn["start"].tolist(), sn["acc"].tolist())))
    assert res[0] == res[1]
    d = b.fire((1 << 63) - 1, [], [], [], [])
    assert b.num_keys() == 0 and len(d["keys"]) > 0


def test_store_insert_hot_cold_split_follows_row_order():
    """An evicted row goes to a cold chunk iff it fired unmodified and no earlier row of the call
    (or the store) made its key hot -- also when the rows are classified by several threads."""
    from mxstream.ops.native import load

    m = load()
    n = 300_000
    k = np.repeat(np.arange(n // 2, dtype=np.int64), 2)      # two rows per key, adjacent
    f = np.ones(n, dtype=np.int64)
    f[1::4] = 0   # keys 0, 2, 4, ...: [fired, unfired] -> first row cold, second hot
    f[2::4] = 0   # keys 1, 3, 5, ...: [unfired, fired] -> both hot
    st_ = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    s = (k * 10).astype(np.int64)
    ones = np.ones_like(k)
    st_.insert(k, s, s + 50, k, ones, f, True)
    assert st_.num_cold_rows() == n // 4
    assert st_.num_sessions() == n
    assert st_.num_keys() == n // 2 + n // 4  # hot keys + cold rows (one per cold key here)


def _slab(cols, R, overflow=0):
    """A pinned-slab image as the GPU eviction's counted copy lays it out: int32 counters
    ([7] rows written, [8] slots evicted) in the first 256 bytes, then six int64 columns of R
    rows each (256-byte aligned)."""
    n = len(cols[0])
    a8 = (R * 8 + 255) & ~255
    buf = np.zeros(256 + 6 * a8, dtype=np.uint8)
    ctr = buf[:64].view(np.int32)
    ctr[7], ctr[8] = n + overflow, n // 2 + 1
    offs = []
    for j, c in enumerate(cols):
        off = 256 + j * a8
        buf[off:off + n * 8].view(np.int64)[:] = c
        offs.append(off)
    return buf, offs


@pytest.mark.parametrize("shards", [1, 4])
def test_store_async_spill_worker_equals_insert(shards):
    """The asynchronous eviction (SessionStore.spill_submit: the persistent C++ worker reads the
    slab, inserts hot rows under the lock, builds the cold chunk outside it, expires) leaves the
    store exactly as the synchronous cold insert + expire_cold: same firings (fire waits only
    for the hot phase), same released keys, same snapshot; a staging overflow keeps only rows
    with cnt > 0."""
    from collections import Counter as Ctr

    from mxstream.ops.native import load

    m = load()
    rng = np.random.default_rng(3)
    a = m.SessionStore(100, 500, K.AGG_SUM_I64, shards)
    b = m.SessionStore(100, 500, K.AGG_SUM_I64, shards)
    keep = []
    got_a, got_b, stats = [], [], {"nr": 0, "ne": 0, "nk": 0}
    for step in range(10):
        n = 2000
        ek = np.sort(rng.integers(step * 1000, step * 1000 + 3000, n)).astype(np.int64)
        es = (step * 400 + (ek % 300)).astype(np.int64)
        acc = (ek % 7).astype(np.int64)
        cnt = np.ones_like(ek)
        flags = np.where(rng.random(n) < 0.9, 1, 0).astype(np.int64)  # 10 % hot rows
        overflow = 5 if step == 4 else 0
        if overflow:
            cnt[::3] = 0  # skipped slots of an overflowed staging buffer
        cols = [ek, es, es + 100, acc, cnt, flags]
        wm = step * 400 - 100
        ok = cnt > 0
        a.insert(*[np.ascontiguousarray(c[ok]) for c in cols], True)
        rel_a = a.expire_cold(wm)
        R = n if overflow else n + 64
        buf, offs = _slab(cols, R, overflow)
        keep.append(buf)
        jid = b.spill_submit(-1, buf.ctypes.data, 0, offs, R, wm)
        assert jid == step + 1
        da = a.fire(step * 400, [], [], [], [], False)
        db = b.fire(step * 400, [], [], [], [], False)
        got_a.append(Ctr(zip(da["keys"].tolist(), da["start"].tolist(), da["raw"].tolist())))
        got_b.append(Ctr(zip(db["keys"].tolist(), db["start"].tolist(), db["raw"].tolist())))
        res = b.spill_join()
        assert [r["id"] for r in res] == [jid]
        r = res[0]
        assert r["nr"] == int(ok.sum()) and r["ne"] == n // 2 + 1
        assert r["nk"] == len(np.unique(ek[ok]))
        # The worker's expiry may run before or after this fire (the fire waits for the hot
        # phase only): a key whose hot sessions the fire cleaned can be reported by both; the
        # keys that left the store are the same.
        assert (set(r["released"].tolist()) | set(db["released"].tolist())
                == set(rel_a.tolist()) | set(da["released"].tolist()))
        assert b.spill_completed() == b.spill_submitted() == jid
    assert got_a == got_b and sum(len(x) for x in got_a) > 0
    sa, sb = a.snapshot(), b.snapshot()
    key = lambda d: sorted(zip(d["key"].tolist(), d["start"].tolist(), d["acc"].tolist(),  # noqa: E731
                               d["cnt"].tolist(), d["flags"].tolist()))
    assert key(sa) == key(sb) and a.num_cold_rows() == b.num_cold_rows() > 0


def test_store_async_spill_poll_and_implicit_join():
    """Results arrive through spill_poll without a wait once the worker is done; every call that
    reads cold rows (here num_keys, extract) joins the worker first."""
    import time as _t

    from mxstream.ops.native import load

    m = load()
    st_ = m.SessionStore(100, 10_000, K.AGG_SUM_I64)
    bufs = []
    total = 0
    for step in range(4):
        k = np.arange(step * 50_000, (step + 1) * 50_000, dtype=np.int64)
        one = np.ones_like(k)
        buf, offs = _slab([k, k, k + 100, k % 5, one, one], len(k))
        bufs.append(buf)
        st_.spill_submit(-1, buf.ctypes.data, 0, offs, len(k))
        total += len(k)
    assert st_.num_keys() == total  # joined
    ex = st_.extract(np.array([7, 50_001], dtype=np.int64), 0, 4)
    assert sorted(ex["key"].tolist()) == [7, 50_001]
    t0 = _t.time()
    res = []
    while len(res) < 4 and _t.time() - t0 < 30:
        res += st_.spill_poll()
    assert [r["id"] for r in res] == [1, 2, 3, 4]
    assert sum(r["nr"] for r in res) == total


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 10_000), gap=st.sampled_from([5, 100, 400]),
       batch=st.sampled_from([1, 64, 1000]), lateness=st.sampled_from([0, 300]),
       nkeys=st.sampled_from([2, 50]))
def test_gpu_sessions_equal_cpu(seed, gap, batch, lateness, nkeys):
    # nkeys=2 with batch 1000: ~500 records per key and step (wave-per-key merge path).
    rng = np.random.default_rng(seed)
    n = 1500 if batch > 1 else 300
    ts = np.sort(rng.integers(0, 30_000, n)) + rng.integers(-400, 400, n)
    events = [(int(k), int(t), int(v)) for k, t, v in
              zip(rng.integers(0, nkeys, n), ts, rng.integers(0, 100, n))]
    a, _ = engine(events, gap, 100, lateness, device="cpu", batch=batch)
    b, op = engine(events, gap, 100, lateness, device="cuda", batch=batch)
    assert a == b


@pytest.mark.gpu
def test_gpu_sessions_overflow_and_spill():
    # > 4 live sessions per key (overflow to the host tier) and a tiny slot table with an
    # aggressive idle threshold (spill of cold keys), against the CPU store.
    rng = np.random.default_rng(3)
    n = 20_000
    ts = np.sort(rng.integers(0, 200_000, n))
    keys = rng.integers(0, 3000, n)
    events = [(int(k), int(t), int(v)) for k, t, v in zip(keys, ts, rng.integers(0, 9, n))]
    b, op = engine(events, 50, 30_000, 5_000, device="cuda", batch=2000, max_load=0.05,
                   idle_spill_ms=2_000, cap_log2=6)
    a2, _ = engine(events, 50, 30_000, 5_000, device="cpu", batch=2000)
    assert a2 == b
    assert op.metrics.spilled_keys > 0 or op.metrics.overflow_keys > 0


@pytest.mark.gpu
def test_gpu_sessions_spill_set_grows_on_device():
    # A 16-entry device spill set must grow (GPU rehash of its live keys, no host rebuild) while
    # keys keep spilling and coming back; results equal the CPU store.
    rng = np.random.default_rng(11)
    n = 20_000
    ts = np.sort(rng.integers(0, 200_000, n))
    keys = rng.integers(0, 3000, n)
    events = [(int(k), int(t), int(v)) for k, t, v in zip(keys, ts, rng.integers(0, 9, n))]
    b, op = engine(events, 50, 30_000, 5_000, device="cuda", batch=2000, max_load=0.05,
                   idle_spill_ms=2_000, cap_log2=6, spill_set_log2=4)
    a2, _ = engine(events, 50, 30_000, 5_000, device="cpu", batch=2000)
    assert a2 == b
    assert op.metrics.spilled_keys > 8 and op.spill_log2 > 4


@pytest.mark.gpu
@pytest.mark.parametrize("promote,rows", [(True, True), (True, False), (False, False)])
def test_gpu_spilled_keys_return_to_hbm(promote, rows, monkeypatch):
    # Keys go idle (spilled to host DRAM with fired sessions inside the lateness), then receive
    # records again: with promotion their sessions come back to HBM slots and the records are
    # folded on the GPU; without it the host store folds them. Both equal the CPU store.
    rng = np.random.default_rng(5)
    events = []
    for rnd in range(6):  # each round: 300 keys active for 20 s, then idle
        base = rnd * 20_000
        for k in range(300):
            for t in rng.integers(base, base + 20_000, 6):
                events.append((k + 300 * (rnd % 2), int(t), int(rng.integers(0, 9))))
    events.sort(key=lambda e: e[1])
    kw = dict(max_load=0.05, idle_spill_ms=3_000, cap_log2=7)
    import mxstream.runtime.session_operator as so

    monkeypatch.setattr(so, "_PROMOTE_ROWS", rows)
    b, op = engine_with(events, 5_000, 2_000, 30_000, promote=promote, device="cuda", batch=600, **kw)
    a2, _ = engine(events, 5_000, 2_000, 30_000, device="cpu", batch=600)
    assert a2 == b
    assert op.metrics.spilled_keys > 0
    if promote:
        assert op.metrics.promoted_keys > 0 and op.metrics.records_promoted > 0
    else:
        assert op.metrics.records_to_host > 0


def engine_with(events, gap, bound, lateness, *, promote, device, batch, **kw):
    op = KeyedSessionOperator(gap=gap, lateness=lateness, agg=K.AGG_SUM_I64, device=device,
                              max_keys=1 << 10, batch_capacity=max(batch, 64), ooo_bound=bound,
                              **kw)
    op.promote_spilled = promote
    out = Counter()
    for i in range(0, len(events), batch):
        chunk = events[i:i + batch]
        k = torch.tensor([e[0] for e in chunk], dtype=torch.int64, device=device)
        t = torch.tensor([e[1] for e in chunk], dtype=torch.int64, device=device)
        v = torch.tensor([e[2] for e in chunk], dtype=torch.int64, device=device)
        for r in (op.process(k, t, v),):
            for kk, s_, e_, rr, c in zip(r.keys, r.start, r.end, r.raw, r.counts):
                out[(int(kk), int(s_), int(e_), int(rr), int(c))] += 1
    r = op.finish()
    for kk, s_, e_, rr, c in zip(r.keys, r.start, r.end, r.raw, r.counts):
        out[(int(kk), int(s_), int(e_), int(rr), int(c))] += 1
    return out, op


def test_store_extract_dense_span_equals_sparse():
    """extract() over a dense key span (bitmap + counting-sort path) returns exactly what the
    sparse path (sort + hash probe / row index) returns for the same sessions under an
    order-preserving key map: rows grouped by key in ascending order, arrival order within a
    key, rows past cleanup dropped."""
    from mxstream.ops.native import load

    m = load()
    rng = np.random.default_rng(21)
    base = rng.permutation(np.arange(1000, 41000, dtype=np.int64))
    k = np.concatenate([base, base[:5000]])  # 5000 keys with two cold rows
    st_ = (k % 5000).astype(np.int64) + np.where(np.arange(len(k)) >= len(base), 2000, 0)
    en = st_ + 100
    acc = np.arange(len(k), dtype=np.int64)
    ones = np.ones_like(k)
    sparse_of = lambda x: x * 1_000_003 + 7  # noqa: E731  (monotone: same key order)
    dense_st = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    sparse_st = m.SessionStore(100, 1000, K.AGG_SUM_I64)
    dense_st.insert(k, st_, en, acc, ones, ones, True)
    sparse_st.insert(sparse_of(k), st_, en, acc, ones, ones, True)
    for rnd in range(3):
        want = rng.choice(np.arange(900, 41100, dtype=np.int64), 3000 + 9000 * rnd)
        a = dense_st.extract(want, 4500, 4)
        b = sparse_st.extract(sparse_of(want), 4500, 4)
        assert np.array_equal(sparse_of(a["key"]), b["key"])
        for c in ("start", "end", "acc", "cnt", "flags"):
            assert np.array_equal(a[c], b[c]), c
        assert np.array_equal(np.sort(sparse_of(a["moved"])), np.sort(b["moved"]))
    assert dense_st.num_keys() == sparse_st.num_keys()


def test_store_extract_hands_back_sessions():
    # Promotion back to HBM (GPU operator) takes keys out of the host store: cold rows and hot
    # sessions of keys with <= max_sess sessions; rows past cleanup are dropped; keys with more
    # sessions stay (their cold rows turn hot).
    from mxstream.ops.native import load

    st = load().SessionStore(100, 1_000, K.AGG_SUM_I64)
    a = lambda *x: np.array(x, dtype=np.int64)  # noqa: E731
    # cold rows (fired, unmodified): key 1 live, key 2 past cleanup at wm=5000, key 3 x3 rows
    st.insert(a(1, 2, 3, 3, 3), a(4000, 0, 4000, 4200, 4400), a(4100, 100, 4100, 4300, 4500),
              a(7, 8, 1, 2, 3), a(1, 1, 1, 1, 1), a(1, 1, 1, 1, 1), True)
    st.process(a(4, 3), a(4800, 4700), a(5, 6), 4000)  # key 4 hot only; key 3 gets a hot session
    assert st.num_keys() >= 4
    ex = st.extract(a(1, 2, 3, 4, 9), 5_000, 2)
    assert ex["key"].tolist() == [1, 4]
    assert ex["acc"].tolist() == [7, 5] and ex["flags"].tolist() == [1, 0]
    assert sorted(ex["moved"].tolist()) == [1, 2, 4, 9]  # 3 has 4 sessions > 2: stays
    assert st.contains(3) and not st.contains(1) and not st.contains(4)
    snap = st.snapshot()
    assert sorted(snap["key"].tolist()) == [3, 3, 3, 3]


# ------------------------------------------------------------------ pipelined step (GPU)
@pytest.mark.gpu
@settings(max_examples=8, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 10_000), gap=st.sampled_from([5, 100, 400]),
       batch=st.sampled_from([64, 1000]), lateness=st.sampled_from([0, 300]))
def test_gpu_pipelined_sessions_equal_cpu(seed, gap, batch, lateness):
    """The pipelined step (a batch's fire and spill run after the next batch's fold is enqueued)
    fires exactly the sessions of the CPU store."""
    rng = np.random.default_rng(seed)
    n = 3000
    ts = np.sort(rng.integers(0, 30_000, n)) + rng.integers(-400, 400, n)
    events = [(int(k), int(t), int(v)) for k, t, v in
              zip(rng.integers(0, 50, n), ts, rng.integers(0, 100, n))]
    a, _ = engine(events, gap, 100, lateness, device="cpu", batch=batch)
    b, op = engine(events, gap, 100, lateness, device="cuda", batch=batch, pipeline=True)
    assert a == b
    assert op._pend is None


@pytest.mark.gpu
@pytest.mark.parametrize("promote", [True, False])
def test_gpu_pipelined_overflow_spill_promote(promote):
    """Overflow runs, idle eviction into the host store, rehash and promotion with the pipelined
    step: equal to the CPU store."""
    rng = np.random.default_rng(3)
    n = 20_000
    ts = np.sort(rng.integers(0, 200_000, n))
    keys = rng.integers(0, 3000, n)
    events = [(int(k), int(t), int(v)) for k, t, v in zip(keys, ts, rng.integers(0, 9, n))]
    b, op = engine_with(events, 50, 30_000, 5_000, promote=promote, device="cuda", batch=2000,
                        max_load=0.05, idle_spill_ms=2_000, cap_log2=6, pipeline=True)
    a2, _ = engine(events, 50, 30_000, 5_000, device="cpu", batch=2000)
    assert a2 == b
    assert op.metrics.spilled_keys > 0 or op.metrics.overflow_keys > 0


@pytest.mark.gpu
def test_gpu_pipelined_redo_steps():
    """Steps the speculative fold must skip (a record far older than the provisional time base,
    a value that needs 24-byte records) take the synchronous path inside the pipeline."""
    rng = np.random.default_rng(8)
    events = []
    for step in range(12):
        for _ in range(300):
            events.append((int(rng.integers(0, 40)), 10_000_000_000 + step * 1000
                           + int(rng.integers(0, 900)), int(rng.integers(0, 9))))
    events[5 * 300 + 7] = (3, 10_000_000_000 - (1 << 31), 4)  # older than wm - 2^30
    events[8 * 300 + 9] = (4, 10_000_008_100, 1 << 40)        # outside int32
    a, _ = engine(events, 200, 100, 1 << 33, device="cpu", batch=300)
    b, op = engine(events, 200, 100, 1 << 33, device="cuda", batch=300, pipeline=True)
    assert a == b
    assert op.metrics.extra.get("tbase_redos", 0) >= 1
    assert op.metrics.extra.get("record_widenings", 0) == 1


@pytest.mark.gpu
def test_gpu_pipelined_snapshot_flushes_pending():
    """A snapshot between steps applies the pending step: the same sessions as the unpipelined
    operator, and the pending fire's rows come with the next call."""
    rng = np.random.default_rng(4)
    ops = [KeyedSessionOperator(gap=100, lateness=0, agg=K.AGG_SUM_I64, device="cuda",
                                max_keys=1 << 10, batch_capacity=512, ooo_bound=50, pipeline=p)
           for p in (False, True)]
    fired = [Counter(), Counter()]
    for step in range(6):
        k = torch.from_numpy(rng.integers(0, 30, 500)).cuda()
        t = torch.from_numpy(np.sort(rng.integers(step * 400, step * 400 + 400, 500))).cuda()
        v = torch.from_numpy(rng.integers(0, 9, 500)).cuda()
        for i, op in enumerate(ops):
            r = op.process(k, t, v)
            fired[i].update(zip(r.keys.tolist(), r.start.tolist(), r.raw.tolist()))
        if step == 3:
            s0, s1 = (sorted(zip(*(op.snapshot()[f].tolist() for f in ("key", "start", "acc"))))
                      for op in ops)
            assert s0 == s1
    for i, op in enumerate(ops):
        r = op.finish()
        fired[i].update(zip(r.keys.tolist(), r.start.tolist(), r.raw.tolist()))
    assert fired[0] == fired[1] and sum(fired[0].values()) > 0


def test_store_worker_expiry_releases_large_chunks():
    """The worker's expiry of big cold chunks (the parallel released-key gather, >= 256K rows)
    releases exactly the keys of the live rows, in row order."""
    from mxstream.ops.native import load

    m = load()
    st_ = m.SessionStore(100, 1_000, K.AGG_SUM_I64)
    n = 300_000
    k = np.arange(n, dtype=np.int64) * 3 + 7
    one = np.ones_like(k)
    cnt = np.where(np.arange(n) % 5 == 0, 0, 1).astype(np.int64)  # some rows already taken
    buf, offs = _slab([k, k % 1000, k % 1000 + 50, k % 11, cnt, one], n)
    st_.spill_submit(-1, buf.ctypes.data, 0, offs, n)
    st_.spill_join()
    buf2, offs2 = _slab([k[:1] + 1, k[:1], k[:1], k[:1], one[:1], one[:1]], 1)
    st_.spill_submit(-1, buf2.ctypes.data, 0, offs2, 1, 10 ** 9)  # expiry at a late watermark
    res = st_.spill_join()
    rel = np.concatenate([r["released"] for r in res])
    live = k[cnt != 0]
    assert np.array_equal(rel[:len(live)], live)
