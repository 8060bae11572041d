"""Keyed rolling state operator: ``keyBy(..).max/min/sum/reduce`` and keyed ValueState counters
with a per-record emission of the post-update value (StreamGroupedReduce semantics,
ComputeCpuMax.java:26; BASELINE config 2 "keyed ValueState counter").

Per micro-batch and rank: partition by key group (window_mode 0) -> RCCL all-to-all ->
rolling pass. GPU: rolling_lookup (HBM hash table insert/find, 64-bit sort keys
slot|src|arrival) -> one radix sort -> rolling_heads -> rolling_scan (one wave per key,
ordered shuffle scan seeded by the stored state, fused filter, compacted rows). CPU: the
sequential twin ``rolling_rows``. Output rows are in per-key arrival order.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from ..ops import expr as E
from ..ops import kernels as K
from ..ops.native import load
from ..parallel.comm import Comm, LocalComm

I64_MIN, I64_MAX = K.I64_MIN, K.I64_MAX


def _next_pow2(x: int) -> int:
    return 1 << max(0, int(x - 1).bit_length())


@dataclass
class RollingRows:
    keys: np.ndarray   # uint64
    values: np.ndarray  # int64 raw (f64 bit pattern for float aggregates; count for COUNT)
    tags: np.ndarray   # int64: src rank << 32 | index in that rank's batch


class KeyedRollingOperator:
    def __init__(self, *, agg: int, device="cpu", comm: Comm | None = None,
                 max_keys: int = 1 << 16, parallelism: int | None = None,
                 max_parallelism: int = 128, batch_capacity: int = 1 << 20,
                 cap_log2: int | None = None, filter_prog: E.Program = E.EMPTY, emit_capacity: int | None = None,
                 count_window: int = 0, dense_keys: bool = False, spill: bool = False,
                 spill_load: float = 0.75, spill_target: float = 0.5):
        """count_window = n > 0: tumbling count windows instead of a rolling aggregate
        (``keyBy(..).countWindow(n)`` with an incremental reduce/aggregate: GlobalWindows +
        PurgingTrigger(CountTrigger(n)), chapter2/README.md:78) -- a row is emitted when a key's
        open window reaches n elements (value = the window's aggregate; for avg the sum, the
        count is n), and the state keeps each key's open window.

        dense_keys: keys are dictionary ids in [0, max_keys) (columnar ingest, device-generated
        ids): the slot IS the key id -- no hash probe. Single-rank GPU sort-free COUNT only.

        spill: keyed state beyond the HBM table lives in host DRAM (RollingSpillStore). Every
        slot records the step that last touched it; when the table's load passes `spill_load`
        after a step, the least recently touched keys move to the host store until the load is
        `spill_target` (the table is rebuilt without them). A batch whose keys include spilled
        ones first promotes them back (their (acc, count) re-inserted into HBM), so every record
        is still folded by the GPU pass in arrival order. The headroom (1 - spill_load) must hold
        one micro-batch's new keys."""
        self.device = K.resolve_device(device)
        self.comm = comm or LocalComm()
        self.world, self.rank = self.comm.world, self.comm.rank
        self.agg = agg
        self.count_window = int(count_window)
        if self.count_window < 0 or self.count_window >= (1 << 31):
            raise ValueError("count window size out of range")
        if agg in (K.AGG_AVG_F64, K.AGG_AVG_I64) and not self.count_window:
            raise ValueError("rolling avg is not a Flink rolling aggregate")
        self.parallelism = parallelism or self.world
        self.max_parallelism = max_parallelism
        self.filter_prog = filter_prog
        from .geometry import state_geometry

        self.dense = bool(dense_keys)
        if self.dense:
            if self.world != 1 or self.device.type != "cuda" or cap_log2 is not None:
                raise ValueError("dense_keys: single-rank GPU rolling state only")
            self.nsub, self.cap_log2 = 1, max(6, int(max_keys - 1).bit_length())
        elif self.world == 1 and cap_log2 is None:
            # One rank: no keyBy buckets or LDS sub-tables to size for (the direct GPU path reads
            # the source columns), so a single table at <= 0.7 load keeps small key spaces small
            # enough for the sort-free LDS counter (rolling_hist: <= 16K slots ~ 11K keys).
            self.nsub, self.cap_log2 = 1, max(6, math.ceil(math.log2((max_keys + 64) / 0.7)))
        else:
            self.nsub, self.cap_log2 = state_geometry(max_keys, self.world, cap_log2)
        cap_log2 = self.cap_log2
        self.nsub_log2 = self.nsub.bit_length() - 1
        self.nslots = self.nsub << cap_log2
        dev = self.device
        self.keys_g = torch.full((self.nslots,), -1, dtype=torch.int64, device=dev)
        self.acc_g = torch.zeros(self.nslots, dtype=torch.int64, device=dev)
        self.cnt_g = torch.zeros(self.nslots, dtype=torch.int32, device=dev)
        self.flags = torch.zeros(4, dtype=torch.int32, device=dev)
        self.spill = bool(spill)
        if self.spill:
            if self.dense:
                raise ValueError("spill: hashed keyed state only (dense ids address the table)")
            if not 0.0 < spill_target < spill_load < 1.0:
                raise ValueError("spill: need 0 < spill_target < spill_load < 1")
            self.spill_load, self.spill_target = float(spill_load), float(spill_target)
            # last touching step per slot (+1 sink entry for hole records)
            self.last_g = torch.zeros(self.nslots + 1, dtype=torch.int64, device=dev)
            self.store = RollingSpillStore(dev)
            self.live_keys = 0
            # GPU: keys in host DRAM as a device hash set (membership probe per batch); the CPU
            # twin tests membership against the store's sorted keys
            self._set = None
            self._set_used = 0
            self._hit = None
            self._nhit = torch.zeros(1, dtype=torch.int32, device=dev)
            self.spill_stats = {"evictions": 0, "spilled_keys": 0, "promoted_keys": 0}
        kgd = [(kg * self.parallelism // max_parallelism) * self.world // self.parallelism
               for kg in range(max_parallelism)]
        self.kg_dest = torch.tensor(kgd, dtype=torch.int32, device=dev)
        self.nbuckets = self.world << self.nsub_log2
        self.stats = K.new_stats(dev)
        self.local_maxts = torch.full((1,), I64_MIN, dtype=torch.int64, device=dev)
        self.red = torch.zeros(K.RED_WORDS, dtype=torch.int64, device=dev)
        self.emit_capacity = emit_capacity
        self._alloc(batch_capacity)
        self.steps = 0
        self.records_in = 0
        self.direct_single_rank = True  # world 1 on the GPU: no partition pass (_process_direct)
        # Sort-free COUNT path (rolling_hist) when the table fits its LDS counter; False forces
        # the sort path (A/B, tests).
        self.sort_free = not self.spill  # the spill tier tracks slots through the sort path
        self._hist_tmp = None
        if self.dense:
            code, consts = filter_prog.as_args()
            if not load().rolling_hist_supported(agg, self.count_window, self.nslots, code, consts):
                raise ValueError("dense_keys: needs the sort-free path (COUNT, no count window, "
                                 "a chain filter, <= 16K keys)")

    def _alloc(self, batch_capacity: int, slack: float = 1.5):
        self.batch_capacity = int(batch_capacity)
        self.slack = slack
        per = self.batch_capacity / self.nbuckets
        nblk = min(1024, max(1, -(-self.batch_capacity // 65536)))
        cap = int(per * slack + 6 * math.sqrt(max(per, 1.0)) + 64) + 8 * nblk
        self.bucket_cap = (cap + 7) & ~7
        words = self.nbuckets * self.bucket_cap * K.REC_WORDS
        dev = self.device
        self.send = torch.empty(words, dtype=torch.int64, device=dev)
        self.recv = torch.empty(words, dtype=torch.int64, device=dev) if self.world > 1 else self.send
        self.cursor = torch.zeros(self.nbuckets, dtype=torch.int32, device=dev)
        self.recv_counts = (torch.zeros(self.nbuckets, dtype=torch.int32, device=dev)
                            if self.world > 1 else self.cursor)
        total = self.nbuckets * self.bucket_cap
        self.sort_key = torch.empty(total, dtype=torch.int64, device=dev)
        self.vals_buf = torch.empty(total, dtype=torch.int64, device=dev)
        self.sort_out = torch.empty(total, dtype=torch.int64, device=dev)
        self.vals_out = torch.empty(total, dtype=torch.int64, device=dev)
        self._sort_tmp = None
        self.heads = torch.empty(total, dtype=torch.int32, device=dev)
        self.n_buf = torch.zeros(2, dtype=torch.int32, device=dev)
        ocap = self.emit_capacity or total
        self.out_key = torch.empty(ocap, dtype=torch.int64, device=dev)
        self.out_val = torch.empty(ocap, dtype=torch.int64, device=dev)
        self.out_tag = torch.empty(ocap, dtype=torch.int64, device=dev)
        # flags[2] is the emitted-row cursor: one D2H returns the row count with the table-full
        # (bit0) and reserved-key (bit2) flags of flags[0].
        self.out_n = self.flags[2:3]

    def _process_direct(self, keys: torch.Tensor, vals: torch.Tensor, n: int, to_host: bool):
        """Single-rank GPU path: every key group is local, so the table lookup reads the source
        columns directly (no partition pass) and writes record i at position i. The batch is then
        in arrival order and a stable radix sort over the slot bits alone gives the (slot,
        arrival) order the scan needs -- the same keys and rows as the partitioned path."""
        m = load()
        st = torch.cuda.current_stream(self.device).cuda_stream
        keys = keys.contiguous()
        vals = vals.contiguous()
        # The kernel reads both columns straight from these pointers: validate like K.partition.
        K._check(keys, torch.int64, n, "keys", self.device)
        K._check(vals, torch.int64, n, "vals", self.device)
        if n >= (1 << 32) or n > self.sort_key.numel():
            raise ValueError("batch larger than the operator's buffers")
        self.records_in += n
        self.steps += 1
        self.out_n.zero_()
        code, consts = self.filter_prog.as_args()
        cap = self.out_key.numel()
        if self.dense or (self.sort_free and m.rolling_hist_supported(
                self.agg, self.count_window, self.nslots, code, consts)):
            # Counting formulation: per-chunk LDS histograms, a cross-chunk prefix seeded by the
            # stored counts, then tile-ranked emission (csrc/rolling_hist_hip.hip) -- no sort.
            need = m.rolling_hist_scratch_bytes(n, self.nslots)
            if self._hist_tmp is None or self._hist_tmp.numel() < need:
                self._hist_tmp = torch.empty(need, dtype=torch.uint8, device=self.device)
            m.gpu_rolling_hist(keys.data_ptr(), n, self.nsub_log2, self.cap_log2,
                               self.keys_g.data_ptr(), self.cnt_g.data_ptr(),
                               self._hist_tmp.data_ptr(), self._hist_tmp.numel(), code, consts,
                               self.out_key.data_ptr(), self.out_val.data_ptr(),
                               self.out_tag.data_ptr(), self.out_n.data_ptr(), cap,
                               self.flags.data_ptr(), int(self.dense), st)
            return self._emit(to_host)
        self.n_buf.zero_()
        shift = max(1, int(n - 1).bit_length())
        m.gpu_rolling_lookup_direct(keys.data_ptr(), vals.data_ptr(), n, self.nsub_log2,
                                    self.cap_log2, self.keys_g.data_ptr(),
                                    self.sort_key.data_ptr(), self.vals_buf.data_ptr(),
                                    self.n_buf.data_ptr(), self.flags.data_ptr(), shift, st)
        if self.spill:
            self._touch_sorted(self.sort_key[:n], shift)
        nbits = shift + self.nslots.bit_length()
        need = m.gpu_sort_pairs_temp_bytes(n, shift, nbits)
        if self._sort_tmp is None or self._sort_tmp.numel() < need:
            self._sort_tmp = torch.empty(need, dtype=torch.uint8, device=self.device)
        m.gpu_sort_pairs(self._sort_tmp.data_ptr(), self._sort_tmp.numel(),
                         self.sort_key.data_ptr(), self.sort_out.data_ptr(),
                         self.vals_buf.data_ptr(), self.vals_out.data_ptr(), n, shift, nbits, st)
        sk = self.sort_out
        n_in = self.n_buf[0:1]
        m.gpu_rolling_heads(sk.data_ptr(), n_in.data_ptr(), n, self.heads.data_ptr(),
                            self.n_buf[1:2].data_ptr(), shift, st)
        m.gpu_rolling_scan(self.agg, sk.data_ptr(), 0, self.vals_out.data_ptr(), n_in.data_ptr(),
                           self.heads.data_ptr(), self.n_buf[1:2].data_ptr(),
                           min(n, self.nslots), self.acc_g.data_ptr(), self.cnt_g.data_ptr(),
                           self.keys_g.data_ptr(), code, consts, self.out_key.data_ptr(),
                           self.out_val.data_ptr(), self.out_tag.data_ptr(),
                           self.out_n.data_ptr(), cap, shift, shift, st, self.count_window)
        return self._emit(to_host)

    def process(self, keys: torch.Tensor, vals: torch.Tensor, to_host: bool = True):
        """Update state with one micro-batch; returns the emitted rows (host) or the device count."""
        if not self.spill:
            return self._process(keys, vals, to_host)
        self._promote(keys)
        out = self._process(keys, vals, to_host)
        if self.device.type != "cuda":
            touched = torch.isin(self.keys_g, keys)
            self.last_g[:self.nslots][touched] = self.steps
        self._maybe_evict()
        return out

    def _process(self, keys: torch.Tensor, vals: torch.Tensor, to_host: bool):
        n = keys.numel()
        if n > self.batch_capacity:
            self._alloc(n, self.slack)
        if ((self.direct_single_rank or self.dense) and self.world == 1
                and self.device.type == "cuda" and n):
            return self._process_direct(keys, vals, n, to_host)
        dummy_ts = self._dummy_ts(n)  # keyed (non-windowed) records carry no timestamp
        while True:
            K.step_begin(self.cursor, self.stats)
            plan = K.PartitionPlan(max_parallelism=self.max_parallelism, nsub_log2=self.nsub_log2,
                                   nranks=self.world, window_mode=0, drop_late=0, hash_mode=0,
                                   bucket_cap=self.bucket_cap, pane=1)
            if n:
                K.partition(keys, dummy_ts, vals, plan, self.kg_dest, self.cursor, self.send,
                            self.stats)
            K.step_finish(self.stats, self.local_maxts, self.red, bound=0, event_mode=True,
                          proc_now=0, flags=self.flags)
            self.red[5] = -n  # the largest batch over ranks sizes the arrival bits of the sort key
            self.comm.allreduce_min_(self.red[3:8])
            if self.world > 1:
                self.comm.all_to_all(self.recv, self.send)
                self.comm.all_to_all(self.recv_counts, self.cursor)
            red = self.red[3:8].tolist()
            if red[3]:
                raise RuntimeError("keyed state table full: a key found no free slot (raise max_keys)")
            if red[4]:
                raise ValueError("key ids -1 and -2 are reserved (the state tables' markers)")
            if red[0]:
                self._alloc(self.batch_capacity, self.slack * 2)
                continue
            break
        self.records_in += n
        self.steps += 1
        self.out_n.zero_()
        m = load()
        code, consts = self.filter_prog.as_args()
        cap = self.out_key.numel()
        if self.device.type == "cuda":
            st = torch.cuda.current_stream(self.device).cuda_stream
            self.n_buf.zero_()
            abits = max(1, int(-red[2] - 1).bit_length())
            shift = abits + max(0, (self.world - 1).bit_length())
            m.gpu_rolling_lookup(self.recv.data_ptr(), self.recv_counts.data_ptr(), self.world,
                                 self.nsub, self.bucket_cap, self.cap_log2, self.keys_g.data_ptr(),
                                 self.sort_key.data_ptr(), self.vals_buf.data_ptr(),
                                 self.n_buf.data_ptr(), self.flags.data_ptr(), abits, shift, st)
            total = int(self.n_buf[0].item())
            if total and self.spill:
                self._touch_sorted(self.sort_key[:total], shift)
            if total:
                # Key-value radix sort over the used bits (slot | src | arrival): the values ride
                # along, so the scan reads them in order (no permutation gather).
                nbits = shift + self.nslots.bit_length()
                need = m.gpu_sort_pairs_temp_bytes(total, 0, nbits)
                if self._sort_tmp is None or self._sort_tmp.numel() < need:
                    self._sort_tmp = torch.empty(need, dtype=torch.uint8, device=self.device)
                m.gpu_sort_pairs(self._sort_tmp.data_ptr(), self._sort_tmp.numel(),
                                 self.sort_key.data_ptr(), self.sort_out.data_ptr(),
                                 self.vals_buf.data_ptr(), self.vals_out.data_ptr(), total, 0,
                                 nbits, st)
                sk = self.sort_out
                n_in = self.n_buf[0:1]
                m.gpu_rolling_heads(sk.data_ptr(), n_in.data_ptr(), total,
                                    self.heads.data_ptr(), self.n_buf[1:2].data_ptr(), shift, st)
                m.gpu_rolling_scan(self.agg, sk.data_ptr(), 0,
                                   self.vals_out.data_ptr(), n_in.data_ptr(), self.heads.data_ptr(),
                                   self.n_buf[1:2].data_ptr(), min(total, self.nslots),
                                   self.acc_g.data_ptr(), self.cnt_g.data_ptr(),
                                   self.keys_g.data_ptr(), code, consts, self.out_key.data_ptr(),
                                   self.out_val.data_ptr(), self.out_tag.data_ptr(),
                                   self.out_n.data_ptr(), cap, abits, shift, st,
                                   self.count_window)
        else:
            m.cpu_rolling_rows(self.recv.data_ptr(), self.recv_counts.data_ptr(), self.world,
                               self.nsub, self.bucket_cap, self.cap_log2, self.agg,
                               self.keys_g.data_ptr(), self.acc_g.data_ptr(),
                               self.cnt_g.data_ptr(), self.flags.data_ptr(), code, consts,
                               self.out_key.data_ptr(), self.out_val.data_ptr(),
                               self.out_tag.data_ptr(), self.out_n.data_ptr(), cap,
                               self.count_window)
        return self._emit(to_host)

    # ---- host-DRAM spill tier ------------------------------------------------------------------
    def _touch_sorted(self, sk: torch.Tensor, shift: int) -> None:
        """last_g[slot] = step for every slot of the step's sort keys (slot << shift | ...;
        INT64_MAX holes land on the sink entry). Stream-ordered, no host sync."""
        slot = torch.where(sk == I64_MAX, torch.full_like(sk, self.nslots), sk >> shift)
        self.last_g.index_fill_(0, slot, self.steps)

    def _promote(self, keys: torch.Tensor) -> None:
        """Spilled keys of this batch go back to HBM with their (acc, count) before the pass."""
        if not len(self.store) or not keys.numel():
            return
        if self.device.type == "cuda":
            n = keys.numel()
            if self._hit is None or self._hit.numel() < n:
                self._hit = torch.empty(max(n, 1024), dtype=torch.uint8, device=self.device)
            self._nhit.zero_()
            st = torch.cuda.current_stream(self.device).cuda_stream
            load().gpu_set_probe(self._set.data_ptr(), self._set.numel() - 1, keys.data_ptr(), n,
                                 self._hit.data_ptr(), self._nhit.data_ptr(), st)
            if not int(self._nhit.item()):
                return
            hit = self._hit[:n].bool()
        else:
            hit = torch.isin(keys, self.store.keys_on(self.device))
            if not bool(hit.any()):
                return
        uk = torch.unique(keys[hit])
        if self.device.type == "cuda":
            load().gpu_set_erase(self._set.data_ptr(), self._set.numel() - 1, uk.data_ptr(),
                                 uk.numel(), torch.cuda.current_stream(self.device).cuda_stream)
        acc, cnt = self.store.take(uk.cpu().numpy())
        self._make_room(uk.numel(), protect=keys)
        slots = K.table_insert(uk, self.keys_g, nsub_log2=self.nsub_log2, cap_log2=self.cap_log2)
        if bool((slots < 0).any()):
            raise RuntimeError("keyed state table full while promoting spilled keys "
                               "(lower spill_load or raise max_keys)")
        self.acc_g[slots] = torch.from_numpy(acc).to(self.device)
        self.cnt_g[slots] = torch.from_numpy(cnt.astype(np.int32)).to(self.device)
        self.last_g[slots] = self.steps
        self.live_keys += uk.numel()
        self.spill_stats["promoted_keys"] += uk.numel()

    def _maybe_evict(self) -> None:
        self.live_keys = int((self.keys_g != -1).sum())
        self._make_room(0)

    def _make_room(self, extra: int, protect: torch.Tensor | None = None) -> None:
        """Evict the least recently touched keys when live + extra passes spill_load. Keys in
        `protect` (the batch about to be folded) stay resident."""
        if self.live_keys + extra <= self.spill_load * self.nslots:
            return
        need = self.live_keys + extra - int(self.spill_target * self.nslots)
        valid = self.keys_g != -1
        lg = torch.where(valid, self.last_g[:self.nslots], torch.full_like(self.last_g[:1], I64_MAX))
        if protect is not None:
            lg = torch.where(torch.isin(self.keys_g, protect), torch.full_like(lg, I64_MAX), lg)
        need = max(1, min(need, self.live_keys))
        thr = torch.kthvalue(lg, need).values
        ev = valid & (lg <= thr) & (lg != I64_MAX)
        idx = torch.nonzero(ev).flatten()
        ek = self.keys_g[idx]
        self.store.add(ek.cpu().numpy(), self.acc_g[idx].cpu().numpy(),
                       self.cnt_g[idx].cpu().numpy().astype(np.int64))
        self._set_add(ek)
        keep = torch.nonzero(valid & ~ev).flatten()
        kk, ka = self.keys_g[keep].clone(), self.acc_g[keep].clone()
        kc, kl = self.cnt_g[keep].clone(), self.last_g[keep].clone()
        self.keys_g.fill_(-1)
        self.acc_g.zero_()
        self.cnt_g.zero_()
        self.last_g.zero_()
        if kk.numel():
            slots = K.table_insert(kk, self.keys_g, nsub_log2=self.nsub_log2,
                                   cap_log2=self.cap_log2)
            self.acc_g[slots] = ka
            self.cnt_g[slots] = kc
            self.last_g[slots] = kl
        self.live_keys = kk.numel()
        self.spill_stats["evictions"] += 1
        self.spill_stats["spilled_keys"] += idx.numel()

    def _set_add(self, keys: torch.Tensor) -> None:
        """GPU: add evicted keys to the device set (rebuilt from the store at twice its size,
        dropping tombstones, when live + erased entries would pass half the capacity)."""
        if self.device.type != "cuda" or not keys.numel():
            return
        m = load()
        st = torch.cuda.current_stream(self.device).cuda_stream
        self._set_used += keys.numel()
        if self._set is None or 2 * self._set_used > self._set.numel():
            cap = 1 << max(16, int(4 * len(self.store)).bit_length())
            self._set = torch.full((cap,), -1, dtype=torch.int64, device=self.device)
            allk = self.store.keys_on(self.device)
            m.gpu_set_insert(self._set.data_ptr(), cap - 1, allk.data_ptr(), allk.numel(), st)
            self._set_used = allk.numel()
            return
        m.gpu_set_insert(self._set.data_ptr(), self._set.numel() - 1, keys.data_ptr(),
                         keys.numel(), st)

    def host_bytes(self) -> int:
        return self.store.nbytes() if self.spill else 0

    def check(self) -> int:
        """Host check of the sticky flags (table full, reserved key); returns the last step's
        emitted row count. to_host=False callers (benchmarks) call it at the end."""
        return self._check_flags(self.flags.tolist())

    @staticmethod
    def _check_flags(hf) -> int:
        if hf[0] & 1:
            raise RuntimeError("keyed state table full: a key found no free slot (raise max_keys)")
        if hf[0] & 4:
            raise ValueError("key ids -1 and -2 are reserved (the state tables' markers)")
        if hf[0] & 16:
            raise ValueError("dense keyed state: a key id is outside [0, max_keys)")
        return hf[2]

    def _emit(self, to_host: bool):
        if not to_host:
            return self.out_n
        if self.device.type == "cuda" and self.out_key.numel() % 2 == 0:
            # One device-counted copy of the emitted rows and the sticky flags into a pinned slab
            # (the copy kernel reads the row count itself) and ONE wait -- instead of a flag read
            # plus three pageable D2H copies, each its own sync. The rows are copied out of the
            # slab (callers may keep them), so the slab is free again at once.
            from .host_rows import CountedHostRows, PinnedSlabPool

            if getattr(self, "_emit_pool", None) is None:
                self._emit_pool = PinnedSlabPool(max_slabs=4)
            hr = CountedHostRows(self._emit_pool, [self.out_key, self.out_val, self.out_tag],
                                 self.out_n, [self.flags])
            hr.wait()
            self._check_flags(hr.fixed(0).tolist())
            k = min(int(hr.fixed(0)[2]), self.out_key.numel())
            cols = hr.columns(k)
            return RollingRows(cols[0].copy().view(np.uint64), cols[1].copy(), cols[2].copy())
        k = min(self.check(), self.out_key.numel())
        return RollingRows(self.out_key[:k].cpu().numpy().copy().view(np.uint64),
                           self.out_val[:k].cpu().numpy().copy(),
                           self.out_tag[:k].cpu().numpy().copy())

    def _dummy_ts(self, n: int) -> torch.Tensor:
        t = getattr(self, "_ts0", None)
        if t is None or t.numel() < n:
            t = torch.zeros(max(n, 1), dtype=torch.int64, device=self.device)
            self._ts0 = t
        return t[:n]

    def state_of(self, key: int):
        """Current (value, count) of a key (host lookup, tests/inspection)."""
        keys = self.keys_g.cpu().numpy()
        idx = np.nonzero(keys == np.int64(key))[0]
        if not len(idx):
            return self.store.get(int(key)) if self.spill else None
        i = int(idx[0])
        return int(self.acc_g[i].item()), int(self.cnt_g[i].item())

    # ---- checkpoint / restore (runtime/checkpoint.py) --------------------------------------
    def owned_key_groups(self) -> tuple[int, int]:
        from .checkpoint import owned_key_groups

        return owned_key_groups(self.rank, self.world, self.parallelism, self.max_parallelism)

    def snapshot_state(self):
        """Per-key ValueState (accumulator, count) grouped by key group."""
        from .checkpoint import OperatorSnapshot

        live = torch.nonzero(self.keys_g != -1).flatten()
        keys = self.keys_g[live].contiguous()
        cols = {"key": keys.cpu().numpy(), "acc": self.acc_g[live].cpu().numpy(),
                "cnt": self.cnt_g[live].cpu().numpy()}
        if self.spill and len(self.store):
            hk, ha, hc = self.store.rows()
            cols = {"key": np.concatenate([cols["key"], hk]),
                    "acc": np.concatenate([cols["acc"], ha]),
                    "cnt": np.concatenate([cols["cnt"], hc.astype(cols["cnt"].dtype)])}
            keys = torch.from_numpy(cols["key"]).to(self.device)
        kg = K.keygroups(keys, max_parallelism=self.max_parallelism).cpu().numpy()
        meta = {"kind": "rolling", "agg": self.agg, "records_in": self.records_in,
                "steps": self.steps, "count_window": self.count_window}
        return OperatorSnapshot(kg, cols, meta)

    def restore_state(self, rows: dict, meta: dict) -> None:
        if meta["agg"] != self.agg or meta.get("count_window", 0) != self.count_window:
            raise ValueError("checkpoint aggregate / count window does not match the operator")
        self.records_in, self.steps = meta["records_in"], meta["steps"]
        self.keys_g.fill_(-1)
        self.acc_g.zero_()
        self.cnt_g.zero_()
        if not len(rows["key"]):
            return
        if self.spill:
            # every key restarts in host DRAM and is promoted when its next record arrives
            self.store.clear()
            self.last_g.zero_()
            self.store.add(np.ascontiguousarray(rows["key"], dtype=np.int64),
                           np.ascontiguousarray(rows["acc"], dtype=np.int64),
                           np.ascontiguousarray(rows["cnt"], dtype=np.int64))
            self.live_keys = 0
            self._set = None
            self._set_add(self.store.keys_on(self.device))
            return
        dev = self.device
        keys = torch.from_numpy(np.ascontiguousarray(rows["key"])).to(dev)
        if self.dense:
            if bool(((keys < 0) | (keys >= self.nslots)).any()):
                raise RuntimeError("restore: a key id does not fit the dense table (raise max_keys)")
            self.keys_g[keys] = keys
            slots = keys
        else:
            slots = K.table_insert(keys, self.keys_g, nsub_log2=self.nsub_log2,
                                   cap_log2=self.cap_log2)
        if bool((slots < 0).any()):
            raise RuntimeError("restore: keyed state does not fit the table (raise max_keys)")
        self.acc_g[slots] = torch.from_numpy(np.ascontiguousarray(rows["acc"])).to(dev)
        self.cnt_g[slots] = torch.from_numpy(np.ascontiguousarray(rows["cnt"])).to(dev)


class RollingSpillStore:
    """Host-DRAM tier of rolling keyed state: (key, acc, count) rows as sorted numpy columns.
    Evictions append (merged into the sorted columns lazily, when a lookup needs them);
    promotions mark rows dead (compacted once half the rows are dead), so a step's promotion
    costs O(promoted keys), not O(store). `keys_on(device)` is the sorted live-key column on the
    device (the CPU twin's membership test), cached until the store changes."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._k = np.zeros(0, np.int64)
        self._a = np.zeros(0, np.int64)
        self._c = np.zeros(0, np.int64)
        self._alive = np.zeros(0, bool)
        self._dead = 0
        self._pending: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []
        self._dev = None

    def __len__(self) -> int:
        return self._k.size - self._dead + sum(p[0].size for p in self._pending)

    def nbytes(self) -> int:
        return 25 * (self._k.size + sum(p[0].size for p in self._pending))

    def clear(self) -> None:
        self.__init__(self.device)

    def add(self, k: np.ndarray, a: np.ndarray, c: np.ndarray) -> None:
        if k.size:
            self._pending.append((np.asarray(k, np.int64), np.asarray(a, np.int64),
                                  np.asarray(c, np.int64)))
            self._dev = None

    def _merge(self) -> None:
        if not self._pending and 2 * self._dead <= self._k.size:
            return
        live = self._alive
        k = np.concatenate([self._k[live]] + [p[0] for p in self._pending])
        a = np.concatenate([self._a[live]] + [p[1] for p in self._pending])
        c = np.concatenate([self._c[live]] + [p[2] for p in self._pending])
        o = np.argsort(k, kind="stable")
        self._k, self._a, self._c = k[o], a[o], c[o]
        self._alive = np.ones(self._k.size, bool)
        self._dead = 0
        self._pending = []

    def keys_on(self, device) -> torch.Tensor:
        self._merge()
        if self._dev is None:
            k = self._k if not self._dead else self._k[self._alive]
            self._dev = torch.from_numpy(np.ascontiguousarray(k)).to(device)
        return self._dev

    def take(self, keys: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """(acc, count) of `keys` (all present and alive), which leave the store."""
        self._merge()
        i = np.searchsorted(self._k, keys)
        if keys.size and (i.max() >= self._k.size or not np.array_equal(self._k[i], keys)
                          or not self._alive[i].all()):
            raise KeyError("rolling spill store: promoted key not present")
        a, c = self._a[i], self._c[i]
        self._alive[i] = False
        self._dead += keys.size
        self._dev = None
        return a, c

    def get(self, key: int):
        self._merge()
        i = int(np.searchsorted(self._k, key))
        if i < self._k.size and self._k[i] == key and self._alive[i]:
            return int(self._a[i]), int(self._c[i])
        return None

    def rows(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        self._merge()
        live = self._alive
        return self._k[live].copy(), self._a[live].copy(), self._c[live].copy()
