"""Device-resident multi-relation graph layout for the HIP kernels.

HBM layout (built once per graph per device, int32 indices, uint8 relation ids):
  CSR by destination   csr_ptr [N+1], csr_idx [E] (source ids), csr_eid [E] (original edge id)
  CSC by source        csc_ptr [N+1], csc_idx [E] (destination ids), csc_eid [E], csc2csr [E]
  relation ids         per e_feat tensor: rel_csr / rel_csc uint8 [E] (0-based = e_feat - 1)
  long-segment plans   segments with > split edges are cut into `chunk`-edge pieces
                       (hub rows of power-law graphs would otherwise serialise one wave)

Edge ids are the caller's (DGL) edge order. Within a row, edges are ordered either
  order="edge"    by edge id (stable sort): the summation order of DGL's own CSR gspmm; or
  order="source"  by the other end's id (ties by edge id): a chunk of a hub row then covers a
                  narrow range of gathered rows, and the plan's chunk schedule (chunks sorted by
                  their first gathered row) makes the chunks in flight at any moment gather
                  overlapping rows, so a row shared by several hubs is fetched from HBM once and
                  hit in L2 / Infinity Cache by the others. Sums change only by rounding order.
"""
import ctypes

import torch

SPLIT = 256      # segments with more edges than this go through the chunked path
CHUNK = 256      # edges per chunk
FANIN = 64       # chunk partials summed per node of the reduction tree


class SegPlan:
    """Long-segment split plan for one orientation (see regnn_spmm_fwd in regnn_hip.h)."""

    @classmethod
    def none(cls):
        """plan of an orientation whose segments are known to be short (no host sync)."""
        plan = cls.__new__(cls)
        plan.split, plan.chunk, plan.n_long = 0, CHUNK, 0
        plan.long_ids = plan.chunk_long = plan.chunk_off = None
        plan.n_chunk = plan.n_levels = plan.partial_rows = 0
        plan.level_sb, plan.level_desc = None, None
        return plan

    def __init__(self, ptr, split=SPLIT, chunk=CHUNK, idx=None):
        """idx given (rows sorted by gathered id): chunks are scheduled by their first gathered
        row (chunk_sched); kernels take the schedule as chunk_long's second half, split < 0."""
        self.chunk_sched = None
        deg = (ptr[1:] - ptr[:-1]).to(torch.int64)
        long_ids = torch.nonzero(deg > split).flatten()
        self.split, self.chunk = split, chunk
        self.n_long = int(long_ids.numel())
        if self.n_long == 0:
            self.split = 0
            self.long_ids = self.chunk_long = self.chunk_off = None
            self.n_chunk = self.n_levels = self.partial_rows = 0
            self.level_sb, self.level_desc = None, None
            return
        nch = (deg[long_ids] + chunk - 1) // chunk
        self.long_ids = long_ids.to(torch.int32)
        off = torch.cat([nch.new_zeros(1), torch.cumsum(nch, 0)])
        self.chunk_off = off.to(torch.int32)
        self.chunk_long = torch.repeat_interleave(
            torch.arange(self.n_long, device=ptr.device, dtype=torch.int32), nch)
        self.n_chunk = int(off[-1].item())
        self._tree(nch, off)
        if idx is not None:
            l = self.chunk_long.to(torch.int64)
            k = torch.arange(self.n_chunk, device=ptr.device) - off[l]
            first = ptr.to(torch.int64)[long_ids[l]] + k * chunk
            order = torch.sort(idx[first].to(torch.int64), stable=True)[1]
            self.chunk_sched = torch.cat([self.chunk_long, order.to(torch.int32)]).contiguous()

    def _tree(self, counts, in_off, fanin=FANIN):
        """fixed-order reduction tree over each long segment's chunk partials (<= fanin inputs
        per node): level k turns partial rows [sb[p], sb[p+1]) into row base_k + p."""
        dev = counts.device
        rows = torch.arange(self.n_long, device=dev)
        sbs, desc = [], []
        sb_total, base, total_in = 0, self.n_chunk, self.n_chunk
        while int(counts.max().item()) > 1:
            n_out = (counts + fanin - 1) // fanin
            out_off = torch.cat([n_out.new_zeros(1), torch.cumsum(n_out, 0)])
            P = int(out_off[-1].item())
            l = torch.repeat_interleave(rows, n_out)
            j = torch.arange(P, device=dev) - out_off[l]
            sb = torch.cat([in_off[l] + j * fanin, in_off.new_tensor([total_in])])
            sbs.append(sb.to(torch.int32))
            desc += [sb_total, P, base]
            sb_total += P + 1
            base += P
            counts, in_off, total_in = n_out, out_off, P
        self.n_levels = len(sbs)
        self.level_sb = torch.cat(sbs).contiguous() if sbs else None
        self.level_desc = (ctypes.c_int64 * max(1, len(desc)))(*desc)
        self.partial_rows = base

    def partial(self, F, device):
        if self.n_chunk == 0:
            return None
        return torch.empty(self.partial_rows, F, dtype=torch.float32, device=device)


def _word_padded(r):
    """uint8 [E] view of a buffer padded to whole 32-bit words (+1 word): the degree kernels read
    relation ids four at a time (aligned words, bytes past the row masked)."""
    buf = torch.zeros(((r.numel() + 3) // 4 + 1) * 4, dtype=torch.uint8, device=r.device)
    buf[:r.numel()] = r
    return buf[:r.numel()]


class CscPrefix:
    """The CSC restricted to edges whose destination is < n (rows kept in their order): the
    backward of an aggregation whose incoming gradient is zero on destination rows >= n (the
    last REGCN layer under the output head, whose loss covers the first n rows) gathers only
    these edges. Every skipped edge would add tab * pre * 0 to its source's sum."""

    def __init__(self, rg, n):
        keep = rg.csc_idx < n
        ck = torch.cat([keep.new_zeros(1, dtype=torch.int64), torch.cumsum(keep, 0)])
        self.n = int(n)
        self.keep = keep
        self.csc_ptr = ck[rg.csc_ptr.to(torch.int64)].to(torch.int32).contiguous()
        self.csc_idx = rg.csc_idx[keep].contiguous()
        self.E = int(self.csc_idx.numel())
        srt = rg.order == "source"
        split, chunk = rg._split
        self.csc_plan = SegPlan(self.csc_ptr, split, chunk, self.csc_idx if srt else None)


class RelPack:
    """Relation ids of one e_feat tensor laid out for both orientations (+ long-row counts)."""

    def __init__(self, rg, e_feat, num_rel=None):
        e = e_feat.to(rg.device).reshape(-1).to(torch.int64)
        if e.numel() != rg.E:
            raise ValueError(f"e_feat has {e.numel()} entries, graph has {rg.E} edges")
        if e.numel():
            lo, hi = int(e.min().item()), int(e.max().item())
            # reference indexes table[e_feat - 1] (layer/REGraphConv.py:61): ids must be 1..R
            if lo < 1 or hi > 256 or (num_rel is not None and hi > num_rel):
                raise ValueError(f"relation ids must lie in [1, {num_rel or 256}], got [{lo}, {hi}]")
        self.max_rel = int(e.max().item()) if e.numel() else 0
        r = (e - 1).to(torch.uint8)
        self.rel_csr = _word_padded(r[rg.csr_eid])
        self.rel_csc = _word_padded(r[rg.csc_eid])
        self._cnt = {}
        self._csc_prefix = {}
        self.rg = rg

    def rel_csc_prefix(self, pre):
        """rel_csc restricted to a CscPrefix's edges (cached per prefix)."""
        r = self._csc_prefix.get(pre.n)
        if r is None:
            r = self._csc_prefix[pre.n] = _word_padded(self.rel_csc[pre.keep])
        return r

    def row_cnt(self, n_rel):
        """[n_dst, n_rel] int16 (read as uint16) relation histogram of every CSR row of at most
        `split` edges, long rows zero (regnn_degree_cnt): static per graph and e_feat, so the
        degree kernels read 2 n_rel bytes per row instead of walking the relation ids."""
        key = ("rows", n_rel)
        if key not in self._cnt:
            rg = self.rg
            deg = (rg.csr_ptr[1:] - rg.csr_ptr[:-1]).to(torch.int64)
            row = torch.repeat_interleave(torch.arange(rg.n_dst, device=rg.device), deg)
            k = row * n_rel + self.rel_csr.to(torch.int64)
            plan = rg.csr_plan
            if plan.n_long:
                # long rows count zero here: drop their edges before the histogram, whose
                # atomics would otherwise serialise on the hub rows' bins
                long_row = torch.zeros(rg.n_dst, dtype=torch.bool, device=rg.device)
                long_row[plan.long_ids.to(torch.int64)] = True
                k = k[~long_row[row]]
            del row
            cnt = torch.bincount(k, minlength=rg.n_dst * n_rel).view(rg.n_dst, n_rel)
            del k
            self._cnt[key] = cnt.to(torch.int16).contiguous()
        return self._cnt[key]

    def long_cnt(self, n_rel):
        """[n_long, n_rel] int32 relation histogram of every long CSR row."""
        plan = self.rg.csr_plan
        if plan.n_long == 0:
            return None
        if n_rel not in self._cnt:
            rg = self.rg
            deg = (rg.csr_ptr[1:] - rg.csr_ptr[:-1]).to(torch.int64)
            lids = plan.long_ids.to(torch.int64)
            row_of = torch.repeat_interleave(torch.arange(plan.n_long, device=rg.device),
                                             deg[lids])
            starts = rg.csr_ptr[lids].to(torch.int64)
            offs = torch.cat([deg.new_zeros(1), torch.cumsum(deg[lids], 0)])[:-1]
            pos = torch.arange(row_of.numel(), device=rg.device) - offs[row_of] + starts[row_of]
            key = row_of * n_rel + self.rel_csr[pos].to(torch.int64)
            # sorted keys + binary search: a histogram would serialise on the hub rows' bins
            key, _ = torch.sort(key)
            bounds = torch.arange(plan.n_long * n_rel + 1, device=rg.device, dtype=key.dtype)
            cnt = torch.diff(torch.searchsorted(key, bounds))
            self._cnt[n_rel] = cnt.view(plan.n_long, n_rel).to(torch.int32).contiguous()
        return self._cnt[n_rel]


class RelGraph:
    """CSR (by destination) + CSC (by source) of a directed multigraph on one device."""

    def __init__(self, src, dst, num_nodes, device, num_dst=None, split=SPLIT, chunk=CHUNK,
                 order="edge"):
        src = torch.as_tensor(src).to(device=device, dtype=torch.int64).reshape(-1)
        dst = torch.as_tensor(dst).to(device=device, dtype=torch.int64).reshape(-1)
        self.device = torch.device(device)
        self.n_src = int(num_nodes)
        self.n_dst = int(num_nodes if num_dst is None else num_dst)
        self.E = int(src.numel())
        if self.E >= 2 ** 31 or max(self.n_src, self.n_dst) >= 2 ** 31:
            raise ValueError("graphs with >= 2^31 edges or nodes need 64-bit offsets (not built)")
        if order not in ("edge", "source"):
            raise ValueError(f"order must be 'edge' or 'source', got {order!r}")
        self.order = order
        if order == "edge":
            _, csr_eid = torch.sort(dst, stable=True)
            _, csc_eid = torch.sort(src, stable=True)
        else:
            _, csr_eid = torch.sort(dst * self.n_src + src, stable=True)
            _, csc_eid = torch.sort(src * self.n_dst + dst, stable=True)
        self.csr_eid = csr_eid
        self.csc_eid = csc_eid
        self.csr_idx = src[csr_eid].to(torch.int32).contiguous()
        self.csc_idx = dst[csc_eid].to(torch.int32).contiguous()
        self.csr_ptr = self._ptr(dst[csr_eid], self.n_dst)
        self.csc_ptr = self._ptr(src[csc_eid], self.n_src)
        inv = torch.empty_like(csr_eid)
        inv[csr_eid] = torch.arange(self.E, device=self.device)
        self.csc2csr = inv[csc_eid].to(torch.int32).contiguous()
        srt = order == "source"
        self.csr_plan = SegPlan(self.csr_ptr, split, chunk, self.csr_idx if srt else None)
        self.csc_plan = SegPlan(self.csc_ptr, split, chunk, self.csc_idx if srt else None)
        self._packs = {}
        self._inv_cnt = None
        self._split = (split, chunk)
        self._prefix = {}

    def csc_prefix(self, n):
        """CscPrefix of the destinations [0, n) (cached; None when it would keep every edge)."""
        n = int(n)
        if n >= self.n_dst:
            return None
        pre = self._prefix.get(n)
        if pre is None:
            if len(self._prefix) > 2:
                self._prefix.clear()
            pre = self._prefix[n] = CscPrefix(self, n)
        return pre

    def _ptr(self, sorted_keys, n):
        # row offsets by binary search over the sorted keys: a histogram (bincount) serialises
        # on the hub rows' atomics (~230 ms per call at mag-10x, 11 M edges into one row)
        if sorted_keys.numel() and (int(sorted_keys[0]) < 0 or int(sorted_keys[-1]) >= n):
            raise ValueError(f"node ids must lie in [0, {n}), got "
                             f"[{int(sorted_keys[0])}, {int(sorted_keys[-1])}]")
        bounds = torch.arange(n + 1, device=sorted_keys.device, dtype=sorted_keys.dtype)
        return torch.searchsorted(sorted_keys, bounds).to(torch.int32).contiguous()

    def in_degree(self):
        return (self.csr_ptr[1:] - self.csr_ptr[:-1])

    def inv_in_count(self):
        """1 / max(in-count, 1) per destination (torch_scatter 'mean' divisor)."""
        if self._inv_cnt is None:
            self._inv_cnt = (1.0 / self.in_degree().clamp(min=1).to(torch.float32)).contiguous()
        return self._inv_cnt

    def rel_pack(self, e_feat, num_rel=None):
        """RelPack for an e_feat tensor, cached on (storage, version, shape)."""
        key = (e_feat.data_ptr(), getattr(e_feat, "_version", 0), tuple(e_feat.shape),
               str(e_feat.device))
        pack = self._packs.get(key)
        if pack is None:
            if len(self._packs) > 8:
                self._packs.clear()
            pack = RelPack(self, e_feat, num_rel)
            pack._keepalive = e_feat
            self._packs[key] = pack
        return pack
