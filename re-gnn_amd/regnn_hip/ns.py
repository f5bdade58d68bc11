"""Device-resident neighbour-sampled (NS) step for the ogbn-mag path (mag/regnn_ns.py:206-214,
392-420) on MI355X: sampler, block aggregation, model step and optimizer with no host
synchronisation, so one training step is one HIP-graph replay.

* ``DeviceSampler`` — the per-hop sampler (regnn_ns_hop, include/regnn_hip.h) over buffers sized
  by capacity: batch B, then B*(k0+1), B*(k0+1)*(k1+1), ... targets / sources per hop. Counts live
  on the device (``sizes``); every later kernel reads them there.
* ``NSBlock`` — one hop's sampled block in the layout its aggregation reads (CSR by target,
  local ids, self loop last, uint8 relation ids, 1/in-count); RelGraph-compatible for ops.
* ``NSTrainer`` — one rank's data-parallel NS training step (regnn_ns_batch -> hops -> REGNN
  forward / nll / backward -> flat-bucket all-reduce -> Adam), captured in a HIP graph when
  asked. Rank r of W takes global batches r, r+W, ... of the epoch's shared permutation
  (SURVEY.md §8e); every rank runs the same number of steps per epoch.

The sampled indices follow the build's sampler spec (oracle/sampler_oracle.py, bit-exact).
"""
import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib as L
from .profile import enabled as profile_enabled, timed

M64 = (1 << 64) - 1


def _i64(u):
    """an unsigned 64-bit value as the int64 with the same bits."""
    u &= M64
    return u - (1 << 64) if u >= (1 << 63) else u


class NSBlock:
    """A sampled bipartite block (sources = n_id[:n_src], targets = n_id[:n_dst]).

    csr_ptr [n_dst+1] int32, csr_idx [E] local source ids (row v's self loop last), rel [E]
    uint8 0-based relation (edge type; num_edge_types + node type for the loop), pos [E] CSR
    position of the sampled edge in the global graph (-1: loop), row [E] each edge's target row,
    inv [n_dst] 1/(sampled + 1).
    n_dst / n_src / E are host ints: exact sizes (API path) or capacities (device engine)."""

    is_ns_block = True

    def __init__(self, ptr, idx, rel, pos, inv, n_dst, n_src, E, device, row=None):
        self.csr_ptr, self.csr_idx, self.rel, self.pos, self.inv = ptr, idx, rel, pos, inv
        self.row = row
        self.n_dst, self.n_src, self.E = int(n_dst), int(n_src), int(E)
        self.device = device

    def __iter__(self):                     # (edge_index, e_id, size) unpacking of the reference
        return iter((self, None, (self.n_src, self.n_dst)))

    def to(self, device):
        return self


class DeviceSampler:
    """Capacity-sized device sampler over a RelGraph (CSR by destination).

    etype: 0-based edge type per caller edge (mag edge_type), or None (relation 0);
    ntype: node type per global node (self-loop relation num_edge_types + ntype), or None."""

    def __init__(self, rg, sizes, batch_size, etype=None, ntype=None, num_edge_types=0,
                 share=None, share_dedup=None):
        """share: another DeviceSampler over the same graph whose read-only tables (edge and
        node types) and dedup tables are reused (a second pipeline slot: the two never sample
        at the same time, and their dedup stamps never coincide). share_dedup: the sampler whose
        dedup tables to reuse instead (default: share); False: tables of its own (a slot that
        may sample at the same time as share, on another stream)."""
        dev = rg.device
        self.rg, self.device = rg, dev
        self.sizes_k = [int(k) for k in sizes]
        if not self.sizes_k or any(k < 1 or k > 64 for k in self.sizes_k):
            raise ValueError(f"device sampler fan-outs must lie in [1, 64], got {sizes}")
        if len(self.sizes_k) > 6:
            raise ValueError("at most 6 hops")
        self.B = int(batch_size)
        caps = [self.B]
        for k in self.sizes_k:
            caps.append(caps[-1] * (k + 1))
        if caps[-1] >= 2 ** 31:
            raise ValueError(f"sampler capacity {caps[-1]} exceeds int32")
        self.caps = caps
        self.num_edge_types = int(num_edge_types)
        n_nodes = max(rg.n_src, rg.n_dst)
        if share is not None:
            self.etype_csr, self.ntype = share.etype_csr, share.ntype
        elif etype is None:
            self.etype_csr = torch.zeros(rg.E, dtype=torch.uint8, device=dev)
        else:
            et = torch.as_tensor(etype).to(dev).reshape(-1)
            if et.numel() != rg.E:
                raise ValueError(f"etype has {et.numel()} entries, graph has {rg.E} edges")
            self.etype_csr = et[rg.csr_eid].to(torch.uint8).contiguous()
        if share is not None:
            pass
        elif ntype is None:
            self.ntype = torch.zeros(n_nodes, dtype=torch.int32, device=dev)
        else:
            self.ntype = torch.as_tensor(ntype).to(dev).to(torch.int32).contiguous()
        if int(self.num_edge_types) + (int(self.ntype.max().item()) if self.ntype.numel() else 0) > 255:
            raise ValueError("relation ids must fit uint8")
        self.state = torch.zeros(8, dtype=torch.int64, device=dev)
        self.sizes = torch.zeros(16, dtype=torch.int32, device=dev)
        self.n_id = torch.zeros(caps[-1], dtype=torch.int32, device=dev)
        dd = share if share_dedup is None else share_dedup
        if dd:
            # one stamp counter for both: the dedup tables need increasing stamps
            self.g2l, self.first = dd.g2l, dd.first
            if dd.stamp_src is None:
                dd.stamp_src = dd.state[4:5].clone()
            self.stamp_src = dd.stamp_src
        else:
            self.g2l = torch.zeros(n_nodes, dtype=torch.int64, device=dev)
            self.first = torch.full((n_nodes,), -1, dtype=torch.int64, device=dev)
            self.stamp_src = None
        self.hop_bufs, self.blocks = [], []
        for h, k in enumerate(self.sizes_k):
            cd = caps[h]
            ce = cd * (k + 1)
            nt = (ce + 1023) // 1024
            z = lambda n, dt=torch.int32: torch.zeros(n, dtype=dt, device=dev)  # noqa: E731
            # tiles: the CSR de-duplication's nt tile counts and their ticket, then the strided
            # transposed index's own ticket, published stamp and error word (nt + 4); status:
            # the strided de-duplication's look-back too (>= ceil(ce / 1024) tiles)
            self.hop_bufs.append(dict(samp=z(cd * k), spos=z(cd * k), scnt=z(cd), gsrc=z(ce),
                                      flag=z(ce, torch.uint8), tiles=z(nt + 4),
                                      status=z(max((cd + 1023) // 1024, nt), torch.int64)))
            blk = NSBlock(z(cd + 1), z(ce), z(ce, torch.uint8), z(ce),
                          torch.ones(cd, dtype=torch.float32, device=dev), cd, caps[h + 1], ce, dev,
                          row=z(ce))
            blk.state = self.state             # the batch's dropout key (the wide epilogue's)
            self.blocks.append(blk)
        self.local, self.edge_meta = None, [None] * len(self.sizes_k)
        self.meta_fresh = [False] * len(self.sizes_k)
        # sums_fresh[h]: the latest run_hops wrote hop h's layer-0 input sums (typed_sums path)
        self.sums_fresh = [False] * len(self.sizes_k)
        self.csc = [None] * len(self.sizes_k)      # per hop: (cnt, ptr, ent, long) or None
        # strided: every hop's block in the fixed-stride layout (row i at i (k + 1), regnn_ns_hop
        # strided) -- the two-layer fused step's layout; False: the CSR layout the module path,
        # exact_adjs and the PyG-style API read
        self.strided = False
        # meta_only[h]: hop h writes only the edge meta its consumer reads (regnn_ns_hop
        # meta_only: no de-duplication, n_id not extended, sampled blk_idx unwritten)
        self.meta_only = [False] * len(self.sizes_k)
        # typed_sums[h]: hop h (meta-only, strided) also forms layer 0's input sums for the
        # fused step (regnn_ns_hop_typed_sums; FusedStep.enable_pre_sums), or None
        self.typed_sums = [None] * len(self.sizes_k)
        self.hop_strided = [None] * len(self.sizes_k)   # per-hop layout override (run_hops)
        self._csc_jobs = {}
        self._csr_fresh = True

    def enable_edge_meta(self, local_node_idx, hop):
        """also write hop `hop`'s per-edge source node type and table row (regnn_ns_hop's
        optional outputs; what regnn_nsm_step's layer 0 gathers by)."""
        self.local = torch.as_tensor(local_node_idx).to(self.device, torch.int64).contiguous()
        ce = self.blocks[hop].csr_idx.numel()
        self.edge_meta[hop] = (torch.zeros(ce, dtype=torch.int32, device=self.device),
                               torch.zeros(ce, dtype=torch.int64, device=self.device))
        self.meta_fresh[hop] = False          # written by the next run_hops
        return self.edge_meta[hop]

    def index_errors(self):
        """device int32 tensor: per hop the strided transposed index's sticky error word (1: a
        block of regnn_ns_hop's index launch gave up waiting for the publish and placed nothing;
        the index of that batch is incomplete). Reading it is one host sync (check_index)."""
        return torch.stack([b["tiles"][-1] for b in self.hop_bufs])

    def check_index(self):
        """raise if any hop's transposed index reported a failed build (index_errors)."""
        bad = self.index_errors().cpu().tolist()
        if any(bad):
            raise RuntimeError(f"regnn_ns_hop: the transposed index build timed out waiting for "
                               f"its publish (hops {[h for h, v in enumerate(bad) if v]})")

    def enable_csc(self, hop):
        """also build hop `hop`'s transposed index (regnn_ns_hop csc_*: per local source, its
        edges' target row << 8 | relation), what the fused step's transposed pass gathers by."""
        ce = self.blocks[hop].csr_idx.numel()
        if ce > 32768:
            raise ValueError(f"the transposed index needs <= 32768 block edges, got {ce}")
        z = lambda n: torch.zeros(n, dtype=torch.int32, device=self.device)  # noqa: E731
        self.csc[hop] = (z(ce), z(ce + 1), z(ce), z(max(ce + 1, CSC_LONG_INTS)))
        return self.csc[hop]

    # -- the per-step device work ------------------------------------------------------------
    def batch_from_perm(self, perm, rank=0, world=1):
        """regnn_ns_batch: this rank's next targets from the epoch permutation (device int64)."""
        L.call("regnn_ns_batch", L.ptr(perm), perm.numel(), self.B, int(rank), int(world),
               L.ptr(self.state), L.ptr(self.n_id), L.ptr(self.sizes),
               None if self.stamp_src is None else L.ptr(self.stamp_src), L.stream())

    def run_hops(self, meta_only=True, strided=None, csc_stream=None, before_sums=None):
        """every hop of the current batch; meta_only=False runs hops marked meta_only in full
        (a consumer that reads n_id / the local source ids, e.g. the module path); strided=False
        writes the CSR blocks whatever self.strided says (None: self.strided). csc_stream
        (strided): a strided hop's transposed index (and its sampled blk_idx) is built on that
        stream, forked after the hop's de-duplication, while the next hop samples on this one;
        the caller joins it. before_sums: called right before the outer hop's sums launch
        (regnn_ns_hop_typed_sums), e.g. to make it wait on an event."""
        strided = self.strided if strided is None else bool(strided)
        # a hop's own layout (hop_strided[h] not None) wins over the call's: the module path
        # samples its outer hop strided with the input sums while hop 0 stays CSR
        hs = lambda h: strided if self.hop_strided[h] is None else self.hop_strided[h]  # noqa: E731
        rg = self.rg
        deferred = -1
        for h, k in enumerate(self.sizes_k):
            b, blk = self.hop_bufs[h], self.blocks[h]
            sh = hs(h)
            fork = (csc_stream is not None and sh and self.csc[h] is not None and
                    self.edge_meta[h] is None)
            if self._sums_path(h, sh, meta_only):
                if before_sums is not None:
                    before_sums()
                ts = self.typed_sums[h]
                et, eo = self.edge_meta[h]
                with timed("ns_typed_sums"):
                    L.call("regnn_ns_hop_typed_sums", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx),
                           L.ptr(self.etype_csr), L.ptr(self.ntype), self.num_edge_types, k, h,
                           L.ptr(self.state), L.ptr(self.sizes), L.ptr(self.n_id), self.caps[h],
                           L.ptr(b["scnt"]), L.ptr(blk.rel), L.ptr(blk.inv), L.ptr(self.local),
                           L.ptr(et), L.ptr(eo), ts["tables"], ts["T"], ts["K"],
                           L.ptr(ts["s_agg"]), L.ptr(ts["s_w"]), L.ptr(ts["u_self"]),
                           L.ptr(ts["u_rel"]),
                           ctypes.addressof(self._csc_job(h - 1)) if deferred == h - 1 else None,
                           L.stream())
                self.meta_fresh[h] = True
                self.sums_fresh[h] = True
                continue
            self.sums_fresh[h] = False
            # the transposed index of this hop built beside the next hop's sums (one launch)
            defer = (not fork and sh and CSC_FUSE["mode"] != "off" and
                     self.csc[h] is not None and self.edge_meta[h] is None and
                     h + 1 < len(self.sizes_k) and self._sums_path(h + 1, hs(h + 1), meta_only))
            L.call("regnn_ns_hop", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(self.etype_csr),
                   L.ptr(self.ntype), self.num_edge_types, k, h, L.ptr(self.state),
                   L.ptr(self.sizes), L.ptr(self.n_id), self.caps[h], L.ptr(self.g2l),
                   L.ptr(self.first), L.ptr(b["samp"]), L.ptr(b["spos"]), L.ptr(b["scnt"]),
                   L.ptr(b["gsrc"]), L.ptr(b["flag"]), L.ptr(b["tiles"]), L.ptr(b["status"]),
                   L.ptr(blk.csr_ptr),
                   L.ptr(blk.csr_idx), L.ptr(blk.rel), L.ptr(blk.pos), L.ptr(blk.row),
                   L.ptr(blk.inv),
                   *((L.ptr(self.local), L.ptr(self.edge_meta[h][0]), L.ptr(self.edge_meta[h][1]))
                     if self.edge_meta[h] is not None else (None, None, None)),
                   int(meta_only and self.meta_only[h] and self.edge_meta[h] is not None),
                   *((L.ptr(t) for t in self.csc[h]) if self.csc[h] is not None
                     else (None, None, None, None)),
                   2 if fork or defer else int(sh), L.stream())
            deferred = h if defer else -1
            if fork:
                csc_stream.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(csc_stream):
                    self._hop_call(h, k, meta_only, 3)
            self.meta_fresh[h] = self.edge_meta[h] is not None
        # the blocks now hold the CSR layout (readable by exact_adjs / model_blocks) or not
        self._csr_fresh = not strided

    def _sums_path(self, h, strided, meta_only):
        """hop h runs as regnn_ns_hop_typed_sums (the fused step's outer hop with layer 0's sums)"""
        return (self.typed_sums[h] is not None and strided and meta_only and self.meta_only[h]
                and self.edge_meta[h] is not None)

    def _csc_job(self, h):
        """regnn_ns_csc_job of hop h's transposed index (its buffers are fixed: built once)"""
        job = self._csc_jobs.get(h)
        if job is None:
            b, blk = self.hop_bufs[h], self.blocks[h]
            cnt, cptr, cent, clong = self.csc[h]
            job = self._csc_jobs[h] = _NsCscJob(
                h, blk.csr_idx.numel(), L.ptr(b["gsrc"]), L.ptr(self.g2l), L.ptr(blk.csr_idx),
                L.ptr(blk.row), L.ptr(blk.rel), L.ptr(cnt), L.ptr(b["tiles"]), L.ptr(cptr),
                L.ptr(cent), L.ptr(clong))
        return job

    def _hop_call(self, h, k, meta_only, mode):
        rg, b, blk = self.rg, self.hop_bufs[h], self.blocks[h]
        L.call("regnn_ns_hop", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(self.etype_csr),
               L.ptr(self.ntype), self.num_edge_types, k, h, L.ptr(self.state),
               L.ptr(self.sizes), L.ptr(self.n_id), self.caps[h], L.ptr(self.g2l),
               L.ptr(self.first), L.ptr(b["samp"]), L.ptr(b["spos"]), L.ptr(b["scnt"]),
               L.ptr(b["gsrc"]), L.ptr(b["flag"]), L.ptr(b["tiles"]), L.ptr(b["status"]),
               L.ptr(blk.csr_ptr), L.ptr(blk.csr_idx), L.ptr(blk.rel), L.ptr(blk.pos),
               L.ptr(blk.row), L.ptr(blk.inv),
               *((L.ptr(self.local), L.ptr(self.edge_meta[h][0]), L.ptr(self.edge_meta[h][1]))
                 if self.edge_meta[h] is not None else (None, None, None)),
               int(meta_only and self.meta_only[h] and self.edge_meta[h] is not None),
               *((L.ptr(t) for t in self.csc[h]) if self.csc[h] is not None
                 else (None, None, None, None)),
               mode, L.stream())

    def set_seed(self, base_seed, epoch, batch_idx):
        """host-driven batches (the PyG-style iterator): seed words + a fresh dedup stamp."""
        st = self.state.cpu()
        st[0], st[1], st[3] = _i64(int(base_seed)), int(epoch), int(batch_idx)
        if self.stamp_src is not None:
            self.stamp_src += 1
            st[4] = int(self.stamp_src.item())
        else:
            st[4] += 1
        self.state.copy_(st)

    def set_targets(self, targets):
        n = int(targets.numel())
        if n > self.B:
            raise ValueError(f"{n} targets exceed the sampler's batch capacity {self.B}")
        self.n_id[:n].copy_(targets.to(torch.int32))
        self.sizes[0:1].fill_(n)
        self.sizes[8:16].zero_()               # strided hops add their edge counts

    def _check_csr(self, what):
        if self.strided:
            raise RuntimeError(f"{what} reads CSR blocks, but this sampler writes the fused "
                               "step's fixed-stride layout (FusedStep set strided = True); call "
                               "run_hops(strided=False) first and read the blocks before the "
                               "next fused step")

    def model_blocks(self):
        """blocks in the model's layer order (outermost hop first, PyG adjs[::-1])."""
        if self.strided and not self._csr_fresh:
            self._check_csr("model_blocks()")
        return self.blocks[::-1]

    def exact_adjs(self):
        """PyG-style per-hop output at exact sizes (one host sync): [(edge_index [2, M] local
        (src, dst) without self loops, dst-major; e_id; (n_src, n_dst); NSBlock copy)], hop
        order (innermost first)."""
        if self.strided and not self._csr_fresh:
            self._check_csr("exact_adjs()")
        sz = self.sizes.cpu().tolist()
        out = []
        for h in range(len(self.sizes_k)):
            blk = self.blocks[h]
            n_dst, n_src, E = sz[h], sz[h + 1], sz[8 + h]
            ptr = blk.csr_ptr[:n_dst + 1].clone()
            idx, rel, pos = blk.csr_idx[:E].clone(), blk.rel[:E].clone(), blk.pos[:E].clone()
            inv = blk.inv[:n_dst].clone()
            cnt = (ptr[1:] - ptr[:-1]).to(torch.int64)
            dst_all = torch.repeat_interleave(torch.arange(n_dst, device=self.device), cnt)
            keep = pos >= 0
            src_l = idx[keep].to(torch.int64)
            dst_l = dst_all[keep]
            e_id = self.rg.csr_eid[pos[keep].to(torch.int64)]
            eb = NSBlock(ptr, idx, rel, pos, inv, n_dst, n_src, E, self.device)
            out.append((torch.stack([src_l, dst_l]), e_id, (n_src, n_dst), eb, cnt - 1))
        return sz[len(self.sizes_k)], out


_P = ctypes.c_void_p
_MT, _ML = 8, 4


class _NsmParams(ctypes.Structure):
    """regnn_nsm_params (include/regnn_hip.h)."""
    _fields_ = [("n_types", ctypes.c_int32), ("k_in", ctypes.c_int32),
                ("n_layers", ctypes.c_int32), ("n_classes", ctypes.c_int32),
                ("alpha", ctypes.c_float), ("p_drop", ctypes.c_float),
                ("n_rel", ctypes.c_int32 * _ML),
                ("x_tab", _P * _MT), ("lin_w", _P * _MT), ("lin_b", _P * _MT),
                ("conv_w", _P * _ML), ("conv_b", _P * _ML), ("conv_rw", _P * _ML),
                ("ln_w", _P * _ML), ("ln_b", _P * _ML), ("out_w", _P), ("out_b", _P),
                ("g_lin_w", _P * _MT), ("g_lin_b", _P * _MT), ("g_conv_w", _P * _ML),
                ("g_conv_b", _P * _ML), ("g_conv_rw", _P * _ML), ("g_ln_w", _P * _ML),
                ("g_ln_b", _P * _ML), ("g_out_w", _P), ("g_out_b", _P), ("loss", _P),
                ("n_edge_types", ctypes.c_int32), ("rel_slots", ctypes.c_int32),
                ("two_layer", ctypes.c_int32)]


class _NsmWork(ctypes.Structure):
    """regnn_nsm_work (include/regnn_hip.h)."""
    _fields_ = [("state", _P), ("sizes", _P), ("n_id", _P), ("cap", ctypes.c_int32 * (_ML + 1)),
                ("blk_ptr", _P * _ML), ("blk_idx", _P * _ML), ("blk_rel", _P * _ML),
                ("blk_inv", _P * _ML), ("ntype", _P), ("local", _P), ("labels", _P),
                ("wc", _P), ("gwc", _P), ("tabs", _P), ("xs", _P * _ML), ("gxs", _P * _ML),
                ("a", _P * _ML), ("stats", _P * _ML), ("ga", _P * _ML), ("edge_type", _P), ("edge_off", _P),
                ("s_agg", _P), ("s_w", _P), ("z", _P), ("beta", _P), ("nvalid", _P), ("slab", _P),
                ("u_self", _P), ("u_rel", _P), ("p0", _P), ("adam", _P), ("gh1", _P),
                ("csc_ptr0", _P), ("csc_ent0", _P), ("csc_long0", _P),
                ("stride", ctypes.c_int32 * _ML), ("blk_cnt", _P * _ML), ("part", ctypes.c_int32),
                ("hub_acc", _P), ("hub_ticket", _P), ("hub_terms", _P), ("split_finalize", ctypes.c_int32),
                ("pre_sums", ctypes.c_int32)]

# include/regnn_hip.h REGNN_CSC_LONG_*: hub rows of a <= 32768-edge block, their <= 1024-entry
# pieces, and the csc_long buffer holding ids + piece table
_LONG_CAP = 32768 // 17 + 1
_CSC_PIECE = 1024                     # include/regnn_hip.h REGNN_CSC_PIECE (256: measured no faster,
#                                       the two-piece rows' ticket path cost what the split saved)
_MAX_PIECE = 32768 // _CSC_PIECE + _LONG_CAP
CSC_LONG_INTS = ((_LONG_CAP + 2) + 3) // 4 * 4 + 4 * _MAX_PIECE


class _NsCscJob(ctypes.Structure):
    """regnn_ns_csc_job (include/regnn_hip.h)."""
    _fields_ = [("hop", ctypes.c_int32), ("cap_e", ctypes.c_int32), ("gsrc", _P), ("g2l", _P),
                ("blk_idx", _P), ("blk_row", _P), ("blk_rel", _P), ("csc_cnt", _P),
                ("tiles", _P), ("csc_ptr", _P), ("csc_ent", _P), ("csc_long", _P)]


class _NsmAdam(ctypes.Structure):
    """regnn_nsm_adam (include/regnn_hip.h)."""
    _fields_ = [("param", _P), ("exp_avg", _P), ("exp_avg_sq", _P), ("grad_base", _P),
                ("n", ctypes.c_int64), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("grad_scale", ctypes.c_float),
                ("step", _P), ("ticket", _P)]


# regnn_nsm_step's two-layer form (re_nsm2.hip): L = 2 and at most 384 classes (its head's LDS)
TWO_LAYER_MAX_CLASSES = 384


def fused_unsupported(model, x_dict):
    """why regnn_nsm_step cannot run this model (None: it can). The fused step covers the
    reference configuration of mag/regnn_ns.py: model 'regcn', self_loop_type 2, use_norm 'ln',
    no residual, feats_type != 2, hidden 64, equal input widths 64 / 128, <= 8 node types,
    2..4 layers, <= 448 classes."""
    if getattr(model, "model", None) != "regcn" or getattr(model, "feats_type", 3) == 2:
        return "model is not the feats_type-3 regcn"
    if model.self_loop_type != 2:
        return "self_loop_type != 2"
    convs = list(model.convs)
    if not 2 <= len(convs) <= _ML:
        return "2..4 layers"
    for c in convs:
        if c.residual or c.use_norm != "ln" or tuple(c.weight.shape) != (64, 64):
            return "conv needs LayerNorm, no residual, hidden 64"
        if c.relation_weight.numel() > 64 or abs(c.scaling_factor - convs[0].scaling_factor) > 0:
            return "relation table > 64 or mixed scaling factors"
    keys = sorted(x_dict)
    if keys != list(range(len(keys))) or len(keys) > _MT:
        return "x_dict keys must be 0..T-1, T <= 8"
    dims = {int(x_dict[k].shape[1]) for k in keys}
    if len(dims) != 1 or dims.pop() not in (64, 128):
        return "input widths must be equal, 64 or 128"
    K = int(x_dict[keys[0]].shape[1])
    if len(keys) * (K + 1) > 600:              # regnn_nsm_step's composed-map bound
        return f"{len(keys)} node types x input width {K} exceed the fused step's tables"
    if any(x_dict[k].dtype != torch.float32 or not x_dict[k].is_contiguous() for k in keys):
        return "inputs must be contiguous fp32"
    if model.out_lin.weight.shape[0] > 448 or model.out_lin.weight.shape[1] != 64:
        return "out_lin must be 64 -> <= 448"
    return None


# "auto": layer 0's relation-slot mode wherever the graph allows it; "off": the edge pass
# (rel0) always (tests compare the two)
REL_SLOTS = {"mode": "auto"}
# "on": the two-layer fused step's sampler writes its blocks in the fixed-stride layout (no
# row-offset scan, sampling and placement in one launch); "off": the CSR blocks (tests that
# inspect them, and the comparison of the two)
STRIDED = {"mode": "on"}
# "on": a one-rank FlatAdam trainer runs Adam inside the two-layer step's last launch; "off":
# the separate regnn_adam_flat launch (tests compare the two)
FUSED_ADAM = {"mode": "on"}
# "on": the pipelined trainer joins the sampler stream between the step's two parts (before
# layer 0's backward); "off": after the whole step (A/B)
SPLIT_JOIN = {"mode": os.environ.get("REGNN_NS_SPLIT_JOIN", "on")}
# "on": several ranks all-reduce the gradients the two-layer step has final after layer 1's
# transposed pass (early_grad_params, the bucket's head) while layer 0's backward runs on a
# forked stream, the rest after the step; "off" (default): one all-reduce of the whole bucket
# after the step. Measured on one rank with the several-rank structure (REGNN_NS_FORCE_EXCHANGE,
# mag-10x, hidden 64): 127.2 us split against 120.0 unsplit and 115.5 without an exchange -- the
# extra reduction launch and the fork / join cost more than the overlap hides while a
# collective's latency, not its bytes, sets its time
SPLIT_EXCHANGE = {"mode": os.environ.get("REGNN_NS_SPLIT_EXCHANGE", "off")}
# "on" (default): the module path (device blocks) samples the next batch on a second stream while
# the model trains on this one, as the fused step does; "off": in order. At hidden 512, mag-10x:
# round 3 (hipBLASLt GEMMs) 1.045 off / 1.09 on; round 4 (x6 GEMMs, interleaved pairs) 0.771 /
# 0.761 off against 0.757 / 0.756 on; round 5 (three interleaved 300-step pairs) 0.683-0.684
# off against 0.667-0.673 on
MODULE_PIPELINE = {"mode": os.environ.get("REGNN_NS_MODULE_PIPELINE", "on")}
# the module path's sampling lookahead (REGNN_NS_MODULE_AHEAD): 1 -- the next batch sampled beside
# each step, a fork and a join per step (each a marker on the model's queue: ~5 us of queue idle
# apiece in a kernel trace at hidden 512); G > 1 -- the fused engine's lookahead groups (2G slots,
# one fork and one join per group of up to G steps); 8 measured 412.3-412.5 against 416.7-416.8
# us per step for 4 at hidden 512, mag-10x (after this round's other module-path changes)
MODULE_AHEAD = {"n": int(os.environ.get("REGNN_NS_MODULE_AHEAD", "8"))}
# "on": the module path's out_lin + loss as ops.ns_lin_xent (labels, per-row loss and the mean in
# one launch; the loss backward with out_lin's bias gradient in one); "off": out_lin, ns_labels
# and ops.softmax_xent (A/B)
LIN_XENT = {"mode": os.environ.get("REGNN_NS_LIN_XENT", "on")}
# "on": the pipelined fused engine builds hop 0's transposed index on a third stream while hop 1
# samples (regnn_ns_hop strided 2 / 3); "off" (default): in the sampler's own chain. Eager runs
# are fine; capturing the third stream (forked from the sampler's stream, joined back before the
# next batch) segfaults inside torch.cuda.graph's capture_end on this image (ROCm 7.2, torch
# 2.10), so the graphed bench cannot use it
CSC_FORK = {"mode": os.environ.get("REGNN_NS_CSC_FORK", "off")}
# "on": hop 0's transposed index is built by extra workgroups of the outer hop's sums launch
# (regnn_ns_hop_typed_sums csc), beside the sums instead of ahead of them in the sampler's
# chain; "off" (default): its own launch after hop 0's de-duplication. Measured (interleaved,
# 300 steps): 111.1-111.5 us on against 107.7-108.4 off -- the sampler's chain is not what
# bounds the step; its waiting workgroups beside the model's kernels cost more than they save
CSC_FUSE = {"mode": os.environ.get("REGNN_NS_CSC_FUSE", "off")}
# the fused engine's sampling lookahead G: 2G sampler slots, each step samples the batch trained
# G steps later, and a G-step graph trains G slots while the sampler fills the other G on the
# second queue with one fork (the graph's root) and one join (its end) -- instead of a fork and
# a join per step, each a few us of queue idle on the model's chain. G = 1: two slots, the
# next batch sampled during this step and joined before layer 0's backward. Measured at
# mag-10x, hidden 64: 134.7 (G=1) / 129.1 (G=4) / 128.1 (G=8) us per step; 16 slots hold
# 0.9 GiB more HBM than 2.
# Round 5 (one rank, 300-step runs): G = 8 107.4-108.4, 16 106.5-108.3, 32 105.6-106.0 us (a
# fork / join per group). Default: 32 with one rank; 8 with several (every captured group holds
# one RCCL all-reduce per step, and that capture was only rehearsed at 8); REGNN_NS_AHEAD wins.
# Round 6: a timed run starts from an idle GPU (after a synchronisation), and a replay's nodes
# reach the queues only as fast as the host enqueues them, so the first group of a run sets how
# late the sampler's queue starts. With a 4-step lead group (PLAN_ORDER "lead4") the 20-step run
# the driver times measured (6 x 20 steps, medians): G = 32 desc 117.8, G = 32 lead4 114.2,
# G = 8 desc 114.0, G = 16 lead4 109.2-110.4 us per step; 160-step runs 106.0 / 105.4 (G = 32
# desc / lead4) against 106.4 (G = 16 lead4). Default: 16 with one rank (32 slots: half the
# lookahead memory of 32)
AHEAD = {"steps": int(os.environ["REGNN_NS_AHEAD"]) if "REGNN_NS_AHEAD" in os.environ else None}


def default_ahead(world):
    return AHEAD["steps"] if AHEAD["steps"] is not None else (16 if world == 1 else 8)
# "on": inside a lookahead group, the sampler's outer-hop sums launch for the group's batch i
# waits for the end of model step i - 1 (a model -> sampler edge only: the model never waits),
# placing it beside step i's agg0 / head; N (default 2): only every N-th batch (each edge costs a
# marker on the model's queue, ~4 us of idle before the next agg0; 6 x 20-step runs: on 111.0,
# 2 110.1, 4 110.2 us; 160 steps 106.2 / 105.5 / 105.5); "off": the sampler runs free
SUMS_ALIGN = {"mode": os.environ.get("REGNN_NS_SUMS_ALIGN", "2")}
# "on": the module path sizes its GEMMs' split-K for the first batch's live rows (ops.LIVE_HINT:
# ~6 k of the 13312-row capacity at mag-10x, split 2 with a reduce); measured at hidden 512 (3 x
# 20 steps): 578.2 against 563.0 us per step without -- the reduce costs more than the shorter
# k-chains save; off by default (REGNN_NS_GEMM_LIVE_HINT=on)
GEMM_LIVE_HINT = {"mode": os.environ.get("REGNN_NS_GEMM_LIVE_HINT", "off")}
# "on": the module path's outer hop forms layer 0's per-type input sums on the sampler's stream
# (relation slots; NSTrainer._module_pre_sums) and layer 0 reads them; "off": layer 0 gathers the
# sampled raw rows itself (regnn_ns_typed_agg, A/B)
MODULE_PRE_SUMS = {"mode": os.environ.get("REGNN_NS_MODULE_PRESUMS", "on")}
# "on": the module path samples hop 0 in the strided layout too (its last layer's forward reads
# the strided rows, its backward the transposed index); "off": hop 0 in the CSR layout (A/B)
MODULE_STRIDED = {"mode": os.environ.get("REGNN_NS_MODULE_STRIDED", "on")}
# "on": FlatAdam advances its step count with a one-element add and launches regnn_adam_flat
# without its end-of-grid ticket (ticket NULL); "off": the launch advances it behind the ticket
ADAM_PRE_STEP = {"mode": os.environ.get("REGNN_ADAM_PRE_STEP", "on")}
# parallel sampler lanes inside a lookahead group (REGNN_NS_SAMPLER_LANES): L streams, slot s on
# lane s mod L with dedup tables of its own lane (L x 16 B per node of HBM). Measured (round 6):
# L = 1 / 2 / 4 at 20 steps 110.6 / 116.0 / 133.0, at 160 steps 105.3 / 112.4 / 137.9 us per step
# -- more sampler work at once slows the model's kernels more than the shorter sampler chain
# saves; 1 stays
SAMPLER_LANES = {"n": int(os.environ.get("REGNN_NS_SAMPLER_LANES", "1"))}
# "on": the module path's last hop runs meta-only when the model's layer 0 is the typed first
# layer (mag.REGNN.typed_first_layer_ok); "off": the full hop (A/B, tests)
MODULE_LEAN_HOP = {"mode": os.environ.get("REGNN_NS_MODULE_LEAN", "on")}
# "on": the fused step's last sampler hop runs meta-only (no dedup / n_id append); "off": the
# full hop (tests that inspect the outermost n_id / local ids)
LEAN_LAST_HOP = {"mode": "on"}
# "on": with relation slots (K = 128, T <= 4) the fused step's outer hop also forms layer 0's
# per-type input sums (regnn_ns_hop_typed_sums) on the sampler's stream, ahead of the model, and
# agg0 reads them (regnn_nsm_work.pre_sums); "off": agg0 gathers the raw rows itself (A/B, tests)
PRE_SUMS = {"mode": os.environ.get("REGNN_NS_PRE_SUMS", "on")}
# capture order of a lookahead group's launches: "model" (every model step, then every sampler
# batch) or "interleave" (model step i, then sampler batch i): the same dependency edges; measured
# (round 6, 20-step runs) within run-to-run spread of each other, so "model" stays
GROUP_ORDER = {"mode": os.environ.get("REGNN_NS_GROUP_ORDER", "model")}


def relation_slots_ok(sampler, T):
    """regnn_nsm_params.rel_slots: True when every (target type, source type) pair of the graph
    has at most one edge relation (ogbn-mag's typed relations: each edge type joins one source
    type to one target type), so layer 0 may sum its input rows per source type unweighted.
    One pass over the graph's edges, cached on the graph."""
    rg = sampler.rg
    key = ("_regnn_rel_slots", sampler.num_edge_types, T)
    cache = getattr(rg, "_regnn_rel_slots", None)
    if cache is not None and cache[0] == key:
        return cache[1]
    dev = rg.device
    ptr = rg.csr_ptr.to(torch.int64)
    present = torch.zeros(_MT * _MT * 256, dtype=torch.bool, device=dev)
    step = 1 << 26
    for a in range(0, rg.E, step):
        b = min(rg.E, a + step)
        pos = torch.arange(a, b, device=dev)
        dst = torch.searchsorted(ptr, pos, right=True) - 1
        st = sampler.ntype[rg.csr_idx[a:b].to(torch.int64)].to(torch.int64)
        dt = sampler.ntype[dst].to(torch.int64)
        r = sampler.etype_csr[a:b].to(torch.int64)
        ok = (st >= 0) & (st < T) & (dt >= 0) & (dt < T)
        present[((dt * _MT + st) * 256 + r)[ok]] = True
    per_pair = present.view(_MT * _MT, 256).sum(1)
    ok = bool((per_pair <= 1).all().item())
    rg._regnn_rel_slots = (key, ok)
    return ok


class FusedStep:
    """regnn_nsm_step over a DeviceSampler's blocks: the model's forward, nll loss and backward
    in eight launches (two layers), gradients written straight into each parameter's .grad (the
    caller's flat bucket views), loss into `loss`. Keeps every buffer it points the library at."""

    def __init__(self, model, sampler, x_dict, node_type, local_node_idx, y_flat, loss):
        why = fused_unsupported(model, x_dict)
        if why is not None:
            raise ValueError(f"regnn_nsm_step does not cover this model: {why}")
        dev = sampler.device
        self.device = dev
        nl = len(model.convs)
        if len(sampler.sizes_k) != nl:
            raise ValueError(f"{nl} layers need {nl} sampler hops, got {len(sampler.sizes_k)}")
        keys = sorted(x_dict)
        T, K = len(keys), int(x_dict[0].shape[1])
        C = int(model.out_lin.weight.shape[0])
        caps = sampler.caps
        self.keep = []                                 # every tensor the structs point at

        def ptr(t):
            self.keep.append(t)
            return t.data_ptr()

        def grad_ptr(p):
            if p.grad is None:                        # frozen parameter (no_re): scratch
                p_scratch = torch.zeros_like(p)
                return ptr(p_scratch)
            return ptr(p.grad)

        P = self.P = _NsmParams()
        P.n_types, P.k_in, P.n_layers, P.n_classes = T, K, nl, C
        P.alpha = float(model.convs[0].scaling_factor)
        P.p_drop = float(model.dropout) if model.training else 0.0
        for t, k in enumerate(keys):
            lin = model.lins[str(k)]
            P.x_tab[t] = ptr(x_dict[k])
            P.lin_w[t], P.lin_b[t] = ptr(lin.weight), ptr(lin.bias)
            P.g_lin_w[t], P.g_lin_b[t] = grad_ptr(lin.weight), grad_ptr(lin.bias)
        for l, c in enumerate(model.convs):
            P.n_rel[l] = c.relation_weight.numel()
            P.conv_w[l], P.conv_b[l], P.conv_rw[l] = ptr(c.weight), ptr(c.bias), ptr(c.relation_weight)
            P.ln_w[l], P.ln_b[l] = ptr(c.norm.weight), ptr(c.norm.bias)
            P.g_conv_w[l], P.g_conv_b[l] = grad_ptr(c.weight), grad_ptr(c.bias)
            P.g_conv_rw[l] = grad_ptr(c.relation_weight)
            P.g_ln_w[l], P.g_ln_b[l] = grad_ptr(c.norm.weight), grad_ptr(c.norm.bias)
        P.out_w, P.out_b = ptr(model.out_lin.weight), ptr(model.out_lin.bias)
        P.g_out_w, P.g_out_b = grad_ptr(model.out_lin.weight), grad_ptr(model.out_lin.bias)
        P.loss = ptr(loss)

        z = lambda *shape: torch.zeros(*shape, dtype=torch.float32, device=dev)  # noqa: E731
        W = self.W = _NsmWork()
        W.state, W.sizes, W.n_id = ptr(sampler.state), ptr(sampler.sizes), ptr(sampler.n_id)
        for h, c in enumerate(caps):
            W.cap[h] = c
        for h, blk in enumerate(sampler.blocks):
            W.blk_ptr[h], W.blk_idx[h] = ptr(blk.csr_ptr), ptr(blk.csr_idx)
            W.blk_rel[h], W.blk_inv[h] = ptr(blk.rel), ptr(blk.inv)
        W.ntype = ptr(sampler.ntype)
        W.local = ptr(torch.as_tensor(local_node_idx).to(dev, torch.int64).contiguous())
        W.labels = ptr(y_flat.to(dev, torch.int64).contiguous())
        W.wc, W.gwc, W.tabs = ptr(z(T, K + 1, 64)), ptr(z(T, K + 1, 64)), ptr(z(nl, 64))
        for l in range(nl):
            n_src, n_dst = caps[nl - l], caps[nl - 1 - l]
            if l > 0:                                  # layer 0 reads the input tables directly
                W.xs[l], W.gxs[l] = ptr(z(n_src, 64)), ptr(z(n_src, 64))
            if l < nl - 1:
                W.a[l], W.stats[l] = ptr(z(n_dst, 64)), ptr(z(n_dst, 2))
            W.ga[l] = ptr(z(n_dst, 64))
        n0 = caps[nl - 1]
        et, eo = sampler.enable_edge_meta(local_node_idx, nl - 1)
        # layer 0 reads its block's sources by (type, table row) only: the last hop skips the
        # first-seen de-duplication and the local ids nothing here reads
        sampler.meta_only[nl - 1] = LEAN_LAST_HOP["mode"] != "off"
        W.edge_type, W.edge_off = ptr(et), ptr(eo)
        W.s_agg, W.z = ptr(z(n0, T, K)), ptr(z(n0, T, K))
        W.s_w, W.beta = ptr(z(n0, T)), ptr(z(n0, T))
        W.nvalid = ptr(z(1))
        # the two-layer step: layer 0 rows' fixed-point gradient sums and group_input's projection
        self.two_layer = (nl == 2 and C <= TWO_LAYER_MAX_CLASSES and
                          sampler.blocks[0].csr_idx.numel() <= 32768)
        # one decision for the library's slab size and step (regnn_nsm_params.two_layer): a
        # batch whose hop-0 block exceeds the transposed index runs the composed-map form
        P.two_layer = int(self.two_layer)
        if self.two_layer:
            W.p0 = ptr(z(caps[1], 64))
            W.gh1 = ptr(z(caps[0], 64))
            _, cptr, cent, clong = sampler.csc[0] or sampler.enable_csc(0)
            W.csc_ptr0, W.csc_ent0, W.csc_long0 = ptr(cptr), ptr(cent), ptr(clong)
            # exact hub-row sums of layer 1's transposed pass (kept zero between steps)
            W.hub_acc = ptr(torch.zeros(_MAX_PIECE * 64, dtype=torch.int64, device=dev))
            W.hub_ticket = ptr(torch.zeros(_LONG_CAP, dtype=torch.int32, device=dev))
            W.hub_terms = ptr(torch.zeros(3 * 64 + 1, dtype=torch.int64, device=dev))
            # the blocks in the fixed-stride layout: sampling and placement in one launch per hop
            sampler.strided = STRIDED["mode"] != "off"
            if sampler.strided:
                for h, k in enumerate(sampler.sizes_k):
                    W.stride[h] = k + 1
                    W.blk_cnt[h] = ptr(sampler.hop_bufs[h]["scnt"])
        self.adam = None
        P.n_edge_types = int(sampler.num_edge_types)
        P.rel_slots = int(REL_SLOTS["mode"] != "off" and relation_slots_ok(sampler, T))
        if P.rel_slots:
            W.u_self = ptr(z(n0, K))
            W.u_rel = ptr(torch.full((n0, T + 1), -1, dtype=torch.int32, device=dev))
        self.slab = z(_slab_floats(P, caps[0]))
        W.slab = ptr(self.slab)
        self.model, self.sampler, self.n_layers = model, sampler, nl
        # layer 0's parameter-free input sums on the sampler (it runs ahead of the model on its
        # own stream): the outer hop writes them straight into this step's s_agg / s_w / u_self
        # / u_rel and agg0 reads them instead of gathering the raw input rows
        if (PRE_SUMS["mode"] != "off" and self.two_layer and P.rel_slots and K == 128 and
                T <= 4 and sampler.strided and sampler.meta_only[nl - 1] and
                max(sampler.sizes_k) <= 63):
            self._tables = (ctypes.c_void_p * T)(*[x_dict[k].data_ptr() for k in keys])
            sampler.typed_sums[nl - 1] = dict(
                tables=self._tables, T=T, K=K, s_agg=self._buf(W.s_agg), s_w=self._buf(W.s_w),
                u_self=self._buf(W.u_self), u_rel=self._buf(W.u_rel))
            W.pre_sums = 1

    def _buf(self, addr):
        """the kept tensor whose data starts at addr."""
        return next(t for t in self.keep if torch.is_tensor(t) and t.data_ptr() == addr)

    def attach_adam(self, opt, grad_flat):
        """the optimizer step joins the last launch (two-layer step): Adam on each parameter
        element right after its gradient's reduction. opt: FlatAdam over the flat parameter
        bucket whose gradient bucket is grad_flat (every parameter's .grad a view into it)."""
        if not self.two_layer:
            raise ValueError("the fused optimizer needs the two-layer step")
        A = self.adam = _NsmAdam()
        A.param, A.exp_avg, A.exp_avg_sq = opt.p.data_ptr(), opt.m.data_ptr(), opt.v.data_ptr()
        A.grad_base, A.n = grad_flat.data_ptr(), grad_flat.numel()
        A.lr, A.beta1, A.beta2, A.eps = opt.lr, float(opt.betas[0]), float(opt.betas[1]), opt.eps
        A.weight_decay, A.grad_scale = opt.weight_decay, opt.grad_scale
        A.step, A.ticket = opt.step_count.data_ptr(), opt.ticket.data_ptr()
        self.keep.extend([opt.p, opt.m, opt.v, grad_flat, opt.step_count, opt.ticket])
        self.W.adam = ctypes.addressof(A)

    def kernels(self):
        """the kernels one regnn_nsm_step launches, in order (bench.py's roofline label)."""
        if self.two_layer:
            ks = ["agg0", "head", "gather", "bwd0"] + ([] if self.P.rel_slots else ["rel0"])
            return ks + ["finalize+adam" if self.adam is not None else "finalize"]
        ks = ["prep", "agg0"] + ["agg"] * (self.n_layers - 2) + ["head"]
        ks += ["agg_bwd", "post_bwd"] * (self.n_layers - 1)
        ks += ["bwd0_rs" if self.P.rel_slots else "bwd0"]
        ks += [] if self.P.rel_slots else ["rel0"]
        return ks + ["finalize", "chain"]

    def launches(self):
        return len(self.kernels())

    def step(self, part=0):
        """part 0: the whole step; 1 / 2 (two-layer step): agg0 + head + gather / bwd0 +
        finalize, so the caller can order other work (the sampler's join) between them."""
        if part and not self.two_layer:
            raise ValueError("the step splits into parts only in its two-layer form")
        self.W.part = int(part)
        if part == 2:
            with torch.cuda.device(self.device):
                L.call("regnn_nsm_step", ctypes.addressof(self.P), ctypes.addressof(self.W),
                       torch.cuda.current_stream(self.device).cuda_stream)
            return
        if not self.sampler.meta_fresh[self.n_layers - 1]:
            raise RuntimeError("run the sampler's hops after building FusedStep: layer 0 reads the "
                               "per-edge source type / table row they write")
        if self.W.pre_sums and not self.sampler.sums_fresh[self.n_layers - 1]:
            # run_hops(meta_only=False) or run_hops(strided=False) samples the outer hop without
            # its input sums: agg0 / bwd0 would read an earlier batch's
            raise RuntimeError("the sampler's latest batch did not form layer 0's input sums "
                               "(run_hops with meta_only=True and the strided layout, as the "
                               "fused step's sampling does)")
        # train / eval decides the dropout (a captured graph keeps the value it was captured with)
        self.P.p_drop = float(self.model.dropout) if self.model.training else 0.0
        with torch.cuda.device(self.device), timed("nsm_step"):
            L.call("regnn_nsm_step", ctypes.addressof(self.P), ctypes.addressof(self.W),
                   torch.cuda.current_stream(self.device).cuda_stream)


def group_sizes(ahead):
    """the multi-step graph lengths at lookahead `ahead` > 1: ahead, ahead / 2, .., 2."""
    out, m = [], int(ahead)
    while m >= 2:
        out.append(m)
        m //= 2
    return out


# the order of a run's replays (plan_run): "desc" (the longest group first, as the greedy split
# finds them), "asc" (shortest first) or "leadL" (a group of L first, then the rest longest
# first). A replay's nodes reach the GPU queues while the host enqueues them; after an idle GPU
# (every timed run starts after a synchronisation) a short first group starts the sampler's
# queue early while the host enqueues the long groups behind it
PLAN_ORDER = {"mode": os.environ.get("REGNN_NS_PLAN", "lead4")}


def _split(k, ahead):
    """k steps as group lengths, longest first (group_sizes(ahead), ones for the rest)."""
    out = []
    while k > 0:
        m = next((m for m in group_sizes(ahead) if m <= k), 1)
        out.append(m)
        k -= m
    return out


def plan_sizes(k, ahead, order=None):
    """the group lengths plan_run replays for k steps, in order (PLAN_ORDER)."""
    order = order or PLAN_ORDER["mode"]
    sizes = _split(k, ahead)
    if order == "asc":
        return sorted(sizes)
    if order.startswith("lead"):
        lead = int(order[4:])
        if lead in group_sizes(ahead) and k > lead and sizes[0] > lead:
            return [lead] + _split(k - lead, ahead)
    return sizes


def plan_run(cur, k, ahead, n_slots, have=lambda m, start: True, order=None):
    """the replays NSTrainer.run_steps issues for k steps from slot `cur` at lookahead `ahead`
    > 1: [(m, start)], m = 1 for a one-step graph; the captured groups (`have`) of the greedy
    split of k into group lengths, in PLAN_ORDER's order, from wherever cur stands (a group
    without a captured graph runs as one-step graphs)."""
    out = []
    for m in plan_sizes(k, ahead, order):
        if m > 1 and not have(m, cur):
            for _ in range(m):
                out.append((1, cur))
                cur = (cur + 1) % n_slots
            continue
        out.append((m, cur))
        cur = (cur + m) % n_slots
    return out


def warm_walk(ahead, n_slots):
    """the replays capture() runs once each (a graph's first launch is slow), in training order
    from slot 0: for every group length m, n_slots times a group then one single step (the start
    advances by m + 1, odd, so it visits every slot) -- every (m, start) group and every
    one-step graph."""
    out, cur = [], 0
    for m in group_sizes(ahead):
        for _ in range(n_slots):
            out.append((m, cur))
            cur = (cur + m) % n_slots
            out.append((1, cur))
            cur = (cur + 1) % n_slots
    return out


def _capturing(g):
    """capture into g with the thread-local error mode: with several ranks the process group's
    watchdog thread polls the eager all-reduces' events meanwhile, which the global mode counts
    as an illegal call during capture (it invalidates the capture at random)."""
    return torch.cuda.graph(g, capture_error_mode="thread_local")


def early_grad_params(model):
    """the parameters whose gradients the two-layer fused step has final after layer 1's
    transposed pass (regnn_nsm_work.split_finalize: reduced at the end of part 1): out_lin,
    layer 1 (weight, bias, relation table, LayerNorm) and layer 0's conv bias and LayerNorm."""
    c0, c1 = model.convs[0], model.convs[1]
    return [model.out_lin.weight, model.out_lin.bias, c1.weight, c1.bias, c1.relation_weight,
            c1.norm.weight, c1.norm.bias, c0.bias, c0.norm.weight, c0.norm.bias]


def _slab_floats(P, cap0):
    n = int(L._so.regnn_nsm_slab_floats(ctypes.addressof(P), int(cap0)))
    if n <= 0:
        raise RuntimeError("regnn_nsm_slab_floats rejected the parameters")
    return n


class FlatAdam:
    """torch.optim.Adam (mag/regnn_ns.py:495: lr, weight_decay) over one flat parameter bucket
    and its flat gradient bucket, one launch per step (regnn_adam_flat); the step count stays on
    the device, so the step can be captured in a HIP graph."""

    def __init__(self, params_flat, grads_flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0):
        self.p, self.g = params_flat, grads_flat
        self.m = torch.zeros_like(params_flat)
        self.v = torch.zeros_like(params_flat)
        dev = params_flat.device
        self.step_count = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lr, self.betas, self.eps, self.weight_decay = float(lr), betas, float(eps), \
            float(weight_decay)
        # the gradient's factor inside the launch (NSTrainer: 1 / ranks, the DP mean of the
        # SUM all-reduce, with no separate division pass)
        self.grad_scale = 1.0

    def step(self):
        pre = ADAM_PRE_STEP["mode"] != "off"
        if pre:
            # the step count advanced by a one-element add before the launch (capturable),
            # instead of the launch's end-of-grid ticket (regnn_adam_flat with ticket NULL)
            self.step_count.add_(1)
        L.call("regnn_adam_flat", L.ptr(self.p), L.ptr(self.g), L.ptr(self.m), L.ptr(self.v),
               self.p.numel(), self.lr, float(self.betas[0]), float(self.betas[1]), self.eps,
               self.weight_decay, self.grad_scale, L.ptr(self.step_count),
               None if pre else L.ptr(self.ticket), L.stream())


class NSTrainer:
    """One rank's NS training step (mag/regnn_ns.py:392-420) on the device sampler.

    model: mag.REGNN; opt: an optimizer over model.parameters() (Adam(capturable=True) for
    graph capture), or None for FlatAdam over a flat parameter bucket (`adam`: lr, betas, eps,
    weight_decay); train_idx: target nodes (the paper train split); y_global [N, 1] labels.
    The gradients live in one flat fp32 bucket (p.grad are views of it): one RCCL all-reduce
    per step for world > 1 (mag.flat_grad_allreduce's exchange), outside the captured graph.

    pipeline: 2 * ahead sampler slots (AHEAD; the module path: MODULE_AHEAD); while the model trains
    on one slot's batch, the batch `ahead` steps later is sampled into another on a second
    stream (the reference's NeighborSampler prefetches batches with DataLoader workers,
    mag/regnn_ns.py:206-208). Slot s deals global batches as rank + s * world of
    2 * ahead * world and the slots train round robin, so the batch sequence is the
    unpipelined one."""

    def __init__(self, model, opt, rg, sizes, batch_size, train_idx, x_dict, edge_type,
                 node_type, local_node_idx, y_global, num_edge_types, seed=0, rank=0, world=1,
                 shuffle=True, engine="auto", adam=None, pipeline=True):
        self.model, self.opt = model, opt
        dev = rg.device
        self.device, self.rank, self.world = dev, int(rank), int(world)
        self.slots = [DeviceSampler(rg, sizes, batch_size, etype=edge_type, ntype=node_type,
                                    num_edge_types=num_edge_types)]
        self.cur, self._primed, self._trained = 0, False, 0
        self.train_idx = torch.as_tensor(train_idx).to(dev, torch.int64)
        self.perm = self.train_idx.clone()
        self.shuffle, self.seed = shuffle, int(seed)
        self.x_dict, self.node_type, self.local_node_idx = x_dict, node_type, local_node_idx
        self.edge_type = torch.as_tensor(edge_type).to(dev, torch.int64)
        self.y_flat = y_global.reshape(-1).to(dev, torch.int64)
        # the module path hands 'regcn' / self_loop_type 2 the capacity-sized device blocks (no
        # host sync: capturable); every other REGNN conv (regat, regatv2, other self-loop types)
        # gets the PyG-style exact-size adjs and edge types (one host sync per step)
        self._blocks_ok = (getattr(model, "model", None) == "regcn" and
                           getattr(model, "self_loop_type", None) == 2)
        self.params = [p for p in model.parameters() if p.requires_grad]
        # every parameter starts on a 16-byte boundary of the flat buckets (the fused step's
        # finalize sums and steps 4 aligned elements per thread); the pad elements stay zero.
        # Two-layer fused step: the gradients final after layer 1's transposed pass lead the
        # bucket ([0, n_early)), so several ranks all-reduce them while layer 0's backward runs.
        why = fused_unsupported(model, x_dict)
        early = []
        if engine != "module" and why is None and len(model.convs) == 2:
            ids = {id(p) for p in self.params}
            early = [p for p in early_grad_params(model) if id(p) in ids]
        eids = {id(p) for p in early}
        order = early + [p for p in self.params if id(p) not in eids]
        offs, o = {}, 0
        for p in order:
            offs[id(p)] = o
            o += (p.numel() + 3) // 4 * 4
            if p is (early[-1] if early else None):
                self.n_early = o
        if not early:
            self.n_early = 0
        self.offsets = [offs[id(p)] for p in self.params]
        self.flat = torch.zeros(o, dtype=torch.float32, device=dev)
        for p, o in zip(self.params, self.offsets):
            p.grad = self.flat[o:o + p.numel()].view_as(p)
        if opt is None:
            # the parameters become views of one flat bucket too, and one launch updates them
            # all (FlatAdam; `adam` = torch.optim.Adam's keyword arguments)
            self.pflat = torch.zeros_like(self.flat)
            for p, o in zip(self.params, self.offsets):
                self.pflat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.pflat[o:o + p.numel()].view_as(p)
            self.opt = opt = FlatAdam(self.pflat, self.flat, **(adam or {}))
            # the data-parallel mean of the SUM all-reduce, inside Adam's launch: no division
            # pass between the exchange and the update (p.grad holds the rank sum)
            opt.grad_scale = 1.0 / self.world
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        # the module path's backward seed d loss / d loss = 1 (autograd would fill one per step)
        self._loss_seed = torch.ones((), dtype=torch.float32, device=dev)
        # ops.ns_lin_xent's last-workgroup ticket (zero between launches)
        self._xent_ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        # engine: "fused" = regnn_nsm_step (the model's forward / loss / backward in eight HIP
        # launches), "module" = the mag.REGNN autograd path, "auto" = fused where it applies
        if engine == "fused" and why is not None:
            raise ValueError(f"fused NS step unavailable: {why}")
        self.fused = None
        if engine != "module" and why is None:
            self.fused = FusedStep(model, self.slots[0], x_dict, node_type, local_node_idx,
                                   self.y_flat, self.loss)
        # the module path on device blocks (regcn, self-loop type 2): capturable, and pipelined
        # like the fused step (the next batch sampled on a second stream)
        self._module_lean = (self.fused is None and self._blocks_ok and
                             MODULE_LEAN_HOP["mode"] != "off" and
                             getattr(model, "typed_first_layer_ok", lambda _x: False)(x_dict))
        if self.fused is None and self._blocks_ok:
            self._setup_module_slot(self.slots[0])
        # REGNN_NS_PIPELINE=0: no second stream (a profiling aid: every kernel's time alone)
        pipeline = pipeline and os.environ.get("REGNN_NS_PIPELINE", "1") != "0"
        self.pipelined = bool(pipeline) and (self.fused is not None or
                                             (self._blocks_ok and MODULE_PIPELINE["mode"] != "off"))
        # the sampling lookahead (fused engine: default_ahead; the module path: MODULE_AHEAD)
        self.ahead = 1
        if self.pipelined:
            self.ahead = max(1, int(default_ahead(self.world) if self.fused is not None
                                    else MODULE_AHEAD["n"]))
        # parallel sampler lanes (lookahead groups): slot s samples on lane s mod L with that
        # lane's own dedup tables, so L batches of a group sample at the same time on L streams
        self.lanes = (max(1, int(SAMPLER_LANES["n"])) if self.pipelined and self.fused is not None
                      and self.ahead > 1 else 1)
        if self.lanes > 1 and (2 * self.ahead) % self.lanes:
            raise ValueError(f"{self.lanes} sampler lanes must divide the {2 * self.ahead} slots")
        if self.pipelined:
            for j in range(1, 2 * self.ahead):
                lane = j % self.lanes
                self.slots.append(DeviceSampler(
                    rg, sizes, batch_size, num_edge_types=num_edge_types, share=self.slots[0],
                    share_dedup=(False if j == lane else self.slots[lane]) if self.lanes > 1
                    else None))
            if self.fused is not None:
                self.fused_slots = [self.fused] + [
                    FusedStep(model, s, x_dict, node_type, local_node_idx, self.y_flat, self.loss)
                    for s in self.slots[1:]]
            else:
                for s in self.slots[1:]:
                    self._setup_module_slot(s)
            # the sampler's stream; REGNN_NS_SIDE_PRIORITY (-1: high) for A/B runs
            self._side = torch.cuda.Stream(device=dev,
                                           priority=int(os.environ.get("REGNN_NS_SIDE_PRIORITY", "0")))
            self._sides = [self._side] + [torch.cuda.Stream(device=dev)
                                          for _ in range(self.lanes - 1)]
            if self.fused is not None and CSC_FORK["mode"] != "off":
                self._csc = torch.cuda.Stream(device=dev)
        # one rank, FlatAdam, two-layer step: the optimizer runs inside the step's last launch
        # (no all-reduce sits between the backward and the update)
        self.adam_fused = (self.fused is not None and self.fused.two_layer and self.world == 1
                           and isinstance(self.opt, FlatAdam) and FUSED_ADAM["mode"] != "off")
        if self.adam_fused:
            for fs in (self.fused_slots if self.pipelined else [self.fused]):
                fs.attach_adam(self.opt, self.flat)
        self.graphs = None
        self.exchange_in_graph = False         # capture() sets it: the all-reduce is in the graphs
        # tests: all-reduce the bucket even with one rank (the captured-exchange path on one GPU)
        self._force_exchange = False
        # several ranks, two-layer fused step: the bucket's early part is all-reduced between the
        # step's two parts while part 2 runs on a forked stream (split_finalize), the rest after
        self._xsplit = False
        self._comm = None
        # False while the graphs hold no collective (several ranks, the exchange between graphs):
        # the whole bucket then goes in one eager all-reduce after each replay
        self._early_ok = True
        if self.world > 1:
            self._set_exchange_split()
        self.epoch = -1
        self.set_epoch(0)

    def _setup_module_slot(self, s):
        """the module path's per-slot sampler outputs: with the typed first layer
        (mag.REGNN._typed_first_layer) the last hop runs meta-only and layer 0 reads its block
        through the per-edge source type / table row; the last layer (hop 0's block)
        differentiates through a gather over that block's transposed index
        (regnn_ns_spmm_bwd_csc: no float atomics into the source rows' gradient)."""
        if self._module_lean:
            last = len(s.sizes_k) - 1
            et, eo = s.enable_edge_meta(self.local_node_idx, last)
            s.meta_only[last] = True
            blk = s.blocks[last]
            blk.edge_meta, blk.meta_only = (et, eo), True
            self._module_pre_sums(s, last)
        for h, blk in enumerate(s.blocks):
            blk.live_rows = s.sizes[h:h + 1]      # the block's live target rows (device count)
        if s.blocks[0].csr_idx.numel() <= 32768:
            _, cptr, cent, clong = s.csc[0] or s.enable_csc(0)
            b0 = s.blocks[0]
            b0.csc, b0.csc_cap = (cptr, cent, clong, s.sizes, 1), s.caps[1]
            from . import ops as _ops
            # (the layer's backward must take the transposed-index gather: ops._NsSpmm)
            if (MODULE_STRIDED["mode"] != "off" and _ops.NS_CSC["mode"] != "off" and
                    len(s.sizes_k) > 1 and
                    getattr(self.model, "hidden_dim", 0) in _ops._CSC_WIDTHS):
                # hop 0 in the strided layout (sampling + placement in one launch, the one-pass
                # de-duplication, the multi-block transposed index): its forward aggregation
                # reads rows at i S (regnn_ns_spmm_strided_fwd), its backward the index
                s.hop_strided[0] = True
                b0.strided_rows = (s.hop_bufs[0]["scnt"], s.sizes_k[0] + 1)

    def _module_pre_sums(self, s, last):
        """relation slots, 128-wide inputs, <= 4 node types: the module path's outer hop runs as
        the sampler's sums launch (regnn_ns_hop_typed_sums, strided, on the sampler's stream) and
        layer 0 reads the per-type sums (ops.ns_slot_agg) instead of gathering the sampled raw
        rows on the model's stream (mag.REGNN._typed_first_layer); hop 0 stays CSR."""
        tabs = getattr(self.model, "_type_tables", lambda _x: None)(self.x_dict)
        T = len(tabs) if tabs else 0
        if (MODULE_PRE_SUMS["mode"] == "off" or not tabs or T > 4 or
                any(t is None or t.dim() != 2 or t.shape[1] != 128 or not t.is_contiguous() or
                    t.data_ptr() % 16 for t in tabs) or max(s.sizes_k) > 63 or
                not relation_slots_ok(s, T)):
            return
        cap, K, dev = s.caps[last], 128, self.device
        z = lambda *shape: torch.zeros(*shape, dtype=torch.float32, device=dev)  # noqa: E731
        U, cnt, xself = z(cap, T, K), z(cap, T), z(cap, K)
        urel = torch.full((cap, T + 1), -1, dtype=torch.int32, device=dev)
        ptrs = (ctypes.c_void_p * T)(*[t.data_ptr() for t in tabs])
        s.typed_sums[last] = dict(tables=ptrs, T=T, K=K, s_agg=U, s_w=cnt, u_self=xself,
                                  u_rel=urel, keep=tabs)
        s.hop_strided[last] = True
        s.blocks[last].pre_sums = (U, cnt, xself, urel)

    # -- epochs ----------------------------------------------------------------------------------
    def steps_per_epoch(self):
        nb = -(-self.train_idx.numel() // self.sampler.B)
        return -(-nb // self.world)

    def set_epoch(self, epoch):
        """shared per-epoch permutation (every rank draws the same one: NeighborSampler's order)."""
        self.epoch = int(epoch)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed * 1_000_003 + self.epoch)
            order = torch.randperm(self.train_idx.numel(), generator=g).to(self.device)
            self.perm.copy_(self.train_idx[order])
        else:
            self.perm.copy_(self.train_idx)
        for s in self.slots:
            st = s.state
            st[0:1].fill_(_i64(self.seed))
            st[1:2].fill_(self.epoch)
            st[2:3].zero_()
        self.cur, self._primed, self._trained = 0, False, 0

    @property
    def sampler(self):
        """the sampler slot of the most recently trained batch."""
        return self.slots[self._trained]

    # -- one step --------------------------------------------------------------------------------
    def _sample(self, slot, before_sums=None):
        n = len(self.slots)
        s = self.slots[slot]
        s.batch_from_perm(self.perm, self.rank + slot * self.world, n * self.world)
        if self.fused is not None:
            # the pipelined engine builds hop 0's transposed index on a third stream while hop 1
            # samples (CSC_FORK), joined back right after: the next batch's sampling writes the
            # dedup tables (g2l) every slot shares, which the index reads
            csc = getattr(self, "_csc", None)
            s.run_hops(csc_stream=csc, before_sums=before_sums)
            if csc is not None:
                torch.cuda.current_stream(self.device).wait_stream(csc)
        else:                                 # the module path reads the CSR blocks
            s.run_hops(meta_only=self._module_lean, strided=False)

    def _pipelined_body(self, cur):
        """train slot `cur`'s batch while the batch of `ahead` steps later is sampled into slot
        cur + ahead (mod 2 ahead; ahead 1: the next batch into the other slot)."""
        cs = torch.cuda.current_stream(self.device)
        nxt = (cur + self.ahead) % len(self.slots)
        self._side.wait_stream(cs)
        if self.fused is None:                # the module path
            self._module_step(self.slots[cur])
            with torch.cuda.stream(self._side):
                self._sample(nxt)
            cs.wait_stream(self._side)
            return
        # the model's launches are issued (captured) before the sampler's: the graph then runs
        # the model chain on the launch queue and the sampler on the second one, and the next
        # replay's first model kernel needs no cross-queue wait (243 -> 234 us per step)
        fs = self.fused_slots[cur]
        # (the profiled eager steps of bench.py time the step as one event: unsplit)
        split = (self.ahead == 1 and fs.two_layer and SPLIT_JOIN["mode"] != "off" and
                 not profile_enabled())
        self._fs_step(fs, part=1 if split else 0)
        with torch.cuda.stream(self._side):
            self._sample(nxt)
        # the join sits between layer 1's transposed pass and layer 0's backward (the sampler is
        # done by then): the next step's first kernel then waits on its own queue only
        cs.wait_stream(self._side)
        if split:
            self._fs_step(fs, part=2)

    def _ahead_group(self, start, m, in_graph):
        """m <= ahead steps from slot `start` as one unit: the model trains slots
        start .. start + m - 1 (sampled earlier: slots cur .. cur + ahead - 1 always are) on the
        launch stream while the sampler fills slots start + ahead .. start + ahead + m - 1 (those
        trained last) on the second one; one fork before, one join after."""
        cs = torch.cuda.current_stream(self.device)
        G, n = self.ahead, len(self.slots)
        for sd in self._sides:
            sd.wait_stream(cs)
        # "on": every step; an integer N: the sums of batches i = N, 2N, .. only (each event
        # record is a marker on the model's queue: ~4 us of queue idle between finalize and the
        # next agg0, measured in a kernel trace); "off": never
        mode = SUMS_ALIGN["mode"]
        every = 0 if mode == "off" or self.fused is None else (1 if mode == "on" else int(mode))
        align = every > 0
        ends = {}

        def model(i):
            if self.fused is None:             # the module path (autograd forward / backward)
                self._module_step(self.slots[(start + i) % n])
            else:
                self._fs_step(self.fused_slots[(start + i) % n])
            if in_graph:
                self._exchange()
            self._opt_step()
            if align and i + 1 < m and (i + 1) % every == 0:
                ev = torch.cuda.Event()
                ev.record(cs)
                ends[i] = ev

        def sampler(i):
            slot = (start + G + i) % n
            sd = self._sides[slot % self.lanes]
            with torch.cuda.stream(sd):
                # batch i's outer-hop sums (the sampler's one heavy launch) wait for the end of
                # model step i - 1, so they run beside step i's agg0 / head (which they slow
                # little) instead of its gather / bwd0 / finalize (2-4x slower beside them)
                wait = ((lambda e=ends[i - 1], sd=sd: sd.wait_event(e))
                        if align and i and (i - 1) in ends else None)
                self._sample(slot, before_sums=wait)

        if GROUP_ORDER["mode"] == "interleave":
            for i in range(m):
                model(i)
                sampler(i)
        else:
            # the model's launches first (captured first: the graph runs them on the launch queue)
            for i in range(m):
                model(i)
            for i in range(m):
                sampler(i)
        for sd in self._sides:
            cs.wait_stream(sd)

    def _group_sizes(self):
        return group_sizes(self.ahead)

    def _advance(self):
        self._trained, self.cur = self.cur, (self.cur + 1) % len(self.slots)

    def _prime(self):
        """the sampled window ahead of slot cur: slots cur .. cur + ahead - 1."""
        if not self._primed:
            for i in range(self.ahead):
                self._sample((self.cur + i) % len(self.slots))
            self._primed = True

    def _forward_backward(self):
        if self.fused is not None:
            # every gradient is overwritten by the step (parameters the forward never reads,
            # e.g. REGNN.norm, keep the zeros of the bucket's allocation)
            if self.pipelined:
                self._prime()
                self._pipelined_body(self.cur)
                self._advance()
                return
            self._sample(0)
            self._fs_step(self.fused)
            return
        if self.pipelined:
            self._prime()
            self._pipelined_body(self.cur)
            self._advance()
            return
        self._trained = 0
        self._sample(0)
        self._module_step(self.slots[0])

    def _module_step(self, s):
        """the mag.REGNN autograd forward / nll / backward on sampler slot s's batch."""
        if (self._blocks_ok and GEMM_LIVE_HINT["mode"] == "on" and
                not getattr(self, "_live_hinted", False) and
                not torch.cuda.is_current_stream_capturing()):
            # the GEMMs' split-K sized for the live rows of a typical block (one host read of
            # the first batch's sizes, eager, before any capture): ops.LIVE_HINT
            from . import ops
            torch.cuda.current_stream(self.device).synchronize()
            sz = s.sizes.cpu().tolist()
            for h in range(1, len(s.caps) - 1):
                ops.set_live_hint(s.caps[h], sz[h])
            self._live_hinted = True
        # the bucket zeroed once: every step overwrites each gradient the forward produces, and
        # a parameter the forward never reads (allow_unused) keeps the zeros (no fill per step)
        if not getattr(self, "_flat_zeroed", False):
            self.flat.zero_()
            self._flat_zeroed = True
        if self._blocks_ok:
            B = s.B
            # the sampler's int32 ids as they are (torch indexes with int32; the HIP ops convert
            # where they need to): no int64 copy per step
            n_id = s.n_id
            from . import mag, ops
            fused_loss = (isinstance(self.model, mag.REGNN) and
                          os.environ.get("REGNN_NS_FUSED_LOSS", "on") != "off")
            ol = getattr(self.model, "out_lin", None)
            lin_xent = (fused_loss and LIN_XENT["mode"] != "off" and ol is not None and
                        getattr(ol, "bias", None) is not None)
            if lin_xent:
                # out_lin, the labels and the loss: ops.ns_lin_xent (forward: the GEMM and one
                # launch; backward: one launch with out_lin's bias gradient, two GEMMs)
                h = self.model(n_id, self.x_dict, s.model_blocks(), None, self.node_type,
                               self.local_node_idx, features=True)
                if h.shape[0] != B:
                    raise RuntimeError(f"the last layer has {h.shape[0]} rows, the batch {B}")
                loss = ops.ns_lin_xent(h, ol.weight, ol.bias, s.n_id, s.sizes, self.y_flat,
                                       self._xent_ticket)
            else:
                out = self.model(n_id, self.x_dict, s.model_blocks(), None, self.node_type,
                                 self.local_node_idx, **({"logits": True} if fused_loss else {}))
                # the targets' labels, -100 (ignored) past the batch's live rows: one launch
                y = ops.ns_labels(s.n_id, s.sizes, self.y_flat, B)
        else:
            # exact sizes (host sync) and the reference's (edge_index, e_id, size) adjs,
            # outermost hop first (mag/regnn_ns.py:399-403)
            n_total, hops = s.exact_adjs()
            adjs = [(ei, e_id, size) for ei, e_id, size, _blk, _cnt in hops[::-1]]
            n_id = s.n_id[:n_total].to(torch.int64)
            out = self.model(n_id, self.x_dict, adjs, self.edge_type, self.node_type,
                             self.local_node_idx)
            y = self.y_flat[n_id[:hops[0][2][1]]]
            fused_loss = lin_xent = False
        if not lin_xent:
            # log_softmax + nll in one launch each way, or the reference's pair (the mean over
            # the batch's targets)
            loss = ops.softmax_xent(out, y) if fused_loss else F.nll_loss(out, y)
        # the gradients straight into the flat bucket: autograd.grad, then one launch copying
        # every gradient (some of them transposed views) into its bucket view (backward() would
        # accumulate with one add kernel per parameter, and _foreach_copy_ / _foreach_add_
        # lower to a kernel per tensor here: ~90 us per step at hidden 512)
        seed = self._loss_seed if loss.shape == self._loss_seed.shape else None
        grads = torch.autograd.grad(loss, self.params, grad_outputs=seed, allow_unused=True)
        # the bucket is zeroed once (above), so a parameter that had a gradient on an earlier
        # step and has none now would keep the stale one: zero exactly those views (the set is
        # the same every step for a fixed model, so this is a host-side set compare only)
        had = getattr(self, "_had_grad", None)
        now = frozenset(i for i, g in enumerate(grads) if g is not None)
        if had is not None and not had <= now:
            with torch.no_grad():
                for i in had - now:
                    self.params[i].grad.zero_()
        self._had_grad = now                  # the views holding a (possibly) non-zero gradient
        with torch.no_grad():
            # (the loss rides in the same launch: no copy of its own)
            dst = [p.grad for p, g in zip(self.params, grads) if g is not None] + [self.loss]
            src = [g for g in grads if g is not None] + [loss.detach()]
            from . import ops
            ops.copy_many(dst, src)

    def _set_exchange_split(self):
        """the split exchange (two-layer fused step without the fused Adam): every slot's step
        reduces the early gradients at the end of its part 1 (regnn_nsm_work.split_finalize)."""
        if (self.fused is None or not self.fused.two_layer or self.adam_fused or
                self.n_early <= 0 or SPLIT_EXCHANGE["mode"] == "off"):
            return
        self._xsplit = True
        self._comm = torch.cuda.Stream(device=self.device)
        for fs in (self.fused_slots if self.pipelined else [self.fused]):
            fs.W.split_finalize = 1

    def _fs_step(self, fs, part=0):
        """the fused step's launches (part 0: both parts); with the split exchange, after part 1
        the early gradients' all-reduce is issued on the launch stream while part 2 runs on a
        forked stream (the collectives stay on the capture's origin stream; the next exchange
        joins the fork)."""
        if not (self._xsplit and self._early_ok):
            fs.step(part=part)
            return
        if part in (0, 1):
            fs.step(part=1)
        if part in (0, 2):
            cs = torch.cuda.current_stream(self.device)
            self._comm.wait_stream(cs)
            self._exchange_early()
            with torch.cuda.stream(self._comm):
                fs.step(part=2)

    def _exchange_early(self):
        import torch.distributed as dist
        dist.all_reduce(self.flat[:self.n_early], op=dist.ReduceOp.SUM)

    def _exchange(self):
        if self.world > 1 or self._force_exchange:
            import torch.distributed as dist
            if self._xsplit and self._early_ok:  # the early part went out after part 1
                torch.cuda.current_stream(self.device).wait_stream(self._comm)
                dist.all_reduce(self.flat[self.n_early:], op=dist.ReduceOp.SUM)
            else:
                dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
            if not isinstance(self.opt, FlatAdam):       # FlatAdam takes the mean itself
                self.flat.div_(self.world)

    def _opt_step(self):
        if not self.adam_fused:                 # else: inside the step's last launch
            self.opt.step()

    def step(self):
        """one eager step (host-launched; no host synchronisation)."""
        self._forward_backward()
        self._exchange()
        self._opt_step()

    def guarded_step(self, guard=None):
        """step() with a failure on any rank ending every rank (regnn_hip.guard): a rank whose
        forward / backward raises still issues the step's gradient all-reduce its peers are in,
        then all ranks agree on the outcome (one eager flag all-reduce) and, if any failed,
        raise guard.RankFailure together. One rank: step()."""
        from .guard import Guard
        guard = guard or Guard(self.world)
        guard.stage("NS train step", self._forward_backward, always=self._exchange)
        self._opt_step()

    def _train_state(self):
        """parameters and optimizer state, for capture() to undo its warm-up steps."""
        if isinstance(self.opt, FlatAdam):
            o = self.opt
            return [t.clone() for t in (o.p, o.m, o.v, o.step_count)], None
        st = {id(p): {k: v.clone() for k, v in s.items() if torch.is_tensor(v)}
              for p, s in self.opt.state.items()}
        return [p.detach().clone() for p in self.params], st

    def _restore_train_state(self, saved):
        flat, st = saved
        with torch.no_grad():
            if st is None:
                o = self.opt
                for dst, src in zip((o.p, o.m, o.v, o.step_count), flat):
                    dst.copy_(src)
                return
            for p, src in zip(self.params, flat):
                p.copy_(src)
            # state tensors the warm-up created (Adam: step, exp_avg, exp_avg_sq) go back to
            # their initial zeros in place: the captured graph keeps their addresses
            for p, s in self.opt.state.items():
                prev = st.get(id(p), {})
                for k, v in s.items():
                    if not torch.is_tensor(v):
                        continue
                    if k in prev:
                        v.copy_(prev[k])
                    else:
                        v.zero_()

    def capture(self, warmup=2, exchange_in_graph=None):
        """capture the step as HIP graphs: [fwd/bwd + optimizer] on one rank; [fwd/bwd] (+ the
        eager all-reduce) + [optimizer] on several. The `warmup` eager steps that precede the
        capture (kernel selection, lazy optimizer state) are undone: parameters, optimizer
        moments and step count, and the sampler's batch / edge counters are restored, so the
        first replay trains the epoch's first batch from the same model as an eager step would.
        Only the dedup stamps move on (they must stay monotone).

        exchange_in_graph (several ranks): the RCCL all-reduce and Adam are captured into the
        step's graph too, so a step is one replay with no host-issued collective and no second
        graph boundary, and runs of steps become one replay per lookahead group as with one rank.
        Default: on with an RCCL ("nccl") process group, off with gloo (a host collective cannot
        be captured); env REGNN_NS_GRAPH_ALLREDUCE=0 / 1 overrides. Measured on one GPU with the
        several-rank structure (rehearse_exchange): 157-160 us per step with the eager exchange
        between graphs, 127 us captured (125.8 one rank). A capture that fails falls back to the
        eager exchange."""
        import os
        multi = self.world > 1 or self._force_exchange
        if exchange_in_graph is None:
            env = os.environ.get("REGNN_NS_GRAPH_ALLREDUCE")
            if env is not None:
                exchange_in_graph = env == "1"
            else:
                import torch.distributed as dist
                exchange_in_graph = (multi and dist.is_available() and dist.is_initialized() and
                                     dist.get_backend() == "nccl")
        if multi and exchange_in_graph:
            saved_state = ([s.state.clone() for s in self.slots], self._train_state())
            err = None
            try:
                # capture only: nothing replays (no collective runs) until every rank agreed
                self._capture(warmup, True, warm=False)
            except RuntimeError as e:          # torch.AcceleratorError is a RuntimeError
                err = e
            # one decision for all ranks, before any replay: a rank replaying graphs with
            # captured all-reduces beside one running eager exchanges would hang the group
            if self._ranks_agree(err is None):
                self._warm_graphs()
                self.exchange_in_graph = True
                return
            import warnings
            why = f"this rank: {err}" if err is not None else "another rank's capture failed"
            warnings.warn(f"capturing the all-reduce into the step graph failed ({why}); every "
                          "rank falls back to the eager exchange between graphs")
            torch.cuda.synchronize(self.device)
            self.graphs, self.graph_groups = None, {}
            self._undo_steps(saved_state[1], saved_state[0])
            exchange_in_graph = False
        self._capture(warmup, bool(exchange_in_graph))
        self.exchange_in_graph = bool(multi and exchange_in_graph)

    def _ranks_agree(self, ok):
        """True when `ok` holds on every rank (an eager MAX all-reduce of the failure flags; one
        rank: ok itself)."""
        import torch.distributed as dist
        if self.world == 1 or not (dist.is_available() and dist.is_initialized()):
            return bool(ok)
        dev = self.device if dist.get_backend() == "nccl" else "cpu"
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return int(flag.item()) == 0

    def _capture(self, warmup, exchange_in_graph, warm=True):
        """the eager warm-up steps (undone), then the graphs; warm: replay every multi-step
        graph once (_warm_graphs) -- capture() defers that until the ranks agreed."""
        multi = self.world > 1 or self._force_exchange
        self._early_ok = not multi or bool(exchange_in_graph)
        if self.fused is None and not self._blocks_ok:
            raise ValueError("this model's module path reads exact-size adjs (a host sync per "
                             "step) and cannot be captured; run step() eagerly")
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        st0 = [s.state.clone() for s in self.slots]
        saved = self._train_state()
        with torch.cuda.stream(side):
            for _ in range(warmup):
                # several ranks: a warm-up step that fails on one rank ends every rank together
                # (regnn_hip.guard) instead of leaving its peers in the step's all-reduce
                if multi:
                    self.guarded_step()
                else:
                    self.step()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self._undo_steps(saved, st0)
        # one rank: the optimizer step joins the step's graph (no graph boundary, no host gap
        # between the backward and Adam); several: the gradient all-reduce runs between graphs,
        # or inside the graph with exchange_in_graph
        fold_opt = not multi or bool(exchange_in_graph)
        in_graph = multi and fold_opt
        if self.pipelined:
            self._prime()                      # slot 0's batch, before the first replay
            torch.cuda.synchronize(self.device)
            g1 = []
            for cur in range(len(self.slots)):   # one graph per slot
                g = torch.cuda.CUDAGraph()
                with _capturing(g):
                    # (Adam after the join: measured faster than before it, the graph then
                    # ends on one queue)
                    self._pipelined_body(cur)
                    if in_graph:
                        self._exchange()
                    if fold_opt:
                        self._opt_step()
                g1.append(g)
            self.graph_groups = {}
            if fold_opt and self.ahead > 1:
                # (m, start) -> m steps from slot start as one graph, m = ahead, ahead / 2, .. 2
                # and every start (run_steps covers any step count from any slot with few
                # replays: a run of k steps takes ~k / ahead graph boundaries and joins)
                for m in self._group_sizes():
                    for start in range(len(self.slots)):
                        g = torch.cuda.CUDAGraph()
                        with _capturing(g):
                            self._ahead_group(start, m, in_graph)
                        self.graph_groups[(m, start)] = g
            elif fold_opt:
                # 2 and 4 steps back to back in one graph (the slot parity returns to 0):
                # run_steps replays them for runs of steps, one graph boundary (~9 us of queue
                # idle between replays) per group instead of per step
                for n in (4, 2):
                    g = torch.cuda.CUDAGraph()
                    with _capturing(g):
                        for i in range(n):
                            self._pipelined_body(i & 1)
                            if in_graph:
                                self._exchange()
                            self._opt_step()
                    self.graph_groups[n] = g
        else:
            g1 = torch.cuda.CUDAGraph()
            with _capturing(g1):
                self._forward_backward()
                if in_graph:
                    self._exchange()
                if fold_opt:
                    self._opt_step()
        g2 = None
        if not fold_opt:
            g2 = torch.cuda.CUDAGraph()
            with _capturing(g2):
                self.opt.step()
        self.graphs = (g1, g2)
        self._cap_undo = (saved, st0, fold_opt)
        if warm:
            self._warm_graphs()

    def _warm_graphs(self):
        """every graph's first launch is slow (tens of us: the runtime's one-time work per
        executable graph); replay each once, walking the slots in training order, and undo those
        steps as the warm-up's (pipelined lookahead groups only)."""
        saved, st0, fold_opt = self._cap_undo
        self._cap_undo = None
        if self.pipelined and fold_opt and self.ahead > 1:
            g1 = self.graphs[0]
            n = len(self.slots)
            for m, start in warm_walk(self.ahead, n):
                assert start == self.cur
                (g1[start] if m == 1 else self.graph_groups[(m, start)]).replay()
                self.cur = (self.cur + m) % n
            self._undo_steps(saved, st0)

    def _undo_steps(self, saved, st0):
        """undo eager or replayed steps taken inside capture(): parameters, optimizer state,
        the sampler's batch and edge counters (not the dedup stamp, state[4]: it stays
        monotone, the tables still hold the undone steps' stamps); slot 0 .. ahead - 1 are
        sampled again by the next step (_prime)."""
        torch.cuda.synchronize(self.device)
        self._restore_train_state(saved)
        for s, s0 in zip(self.slots, st0):
            s.state[2:4].copy_(s0[2:4])
            s.state[5:6].copy_(s0[5:6])
        torch.cuda.synchronize(self.device)
        self.cur, self._primed, self._trained = 0, False, 0

    def run_steps(self, k):
        """k training steps as graph replays (capture() first), the same steps as k replay()s:
        lookahead > 1: the multi-step groups plan_run picks from any slot; lookahead 1: runs of
        4 or 2 steps from slot 0 as one graph, the rest one-step graphs."""
        k = int(k)
        groups = getattr(self, "graph_groups", {})
        if self.ahead > 1:
            n = len(self.slots)
            for m, start in plan_run(self.cur, k, self.ahead, n, lambda m, c: (m, c) in groups):
                if m == 1:
                    self.replay()
                    continue
                self._prime()
                groups[(m, start)].replay()
                self._trained, self.cur = (start + m - 1) % n, (start + m) % n
            return
        while k > 0:
            n = next((n for n in sorted(groups, reverse=True) if n <= k), 0)
            if n and self.cur == 0 and self._primed:
                groups[n].replay()
                self._trained = 1                  # slot 1's batch trained last; cur back to 0
                k -= n
            else:
                self.replay()
                k -= 1

    def replay(self):
        g1, g2 = self.graphs
        if self.pipelined:
            self._prime()                      # after set_epoch: the new epoch's first batch
            g1[self.cur].replay()
            self._advance()
        else:
            g1.replay()
        if g2 is not None:
            self._exchange()
            g2.replay()

    def rehearse_exchange(self):
        """the several-rank step structure on one rank (a timing rehearsal on one GPU, with a
        one-rank process group initialised): the bucket all-reduce after the backward and Adam
        as its own launch after it. Call before capture()."""
        self._force_exchange = True
        if self.adam_fused:
            self.adam_fused = False
            for fs in (self.fused_slots if self.pipelined else [self.fused]):
                fs.adam = None
                fs.W.adam = None
        self._set_exchange_split()

    def param_vector(self):
        """the parameters in model order without the bucket's alignment pads."""
        return torch.cat([p.detach().reshape(-1) for p in self.params])

    def edges_total(self):
        """aggregated edges of every batch sampled so far (device counters: one host sync;
        pipelined, that includes the batch sampled ahead)."""
        # one host sync: the slots' edge counters and (the sampler's own failure report riding
        # on it) every slot's transposed-index error words
        words = torch.cat([torch.stack([s.state[5] for s in self.slots]).sum().reshape(1)] +
                          [s.index_errors().to(torch.int64) for s in self.slots]).cpu().tolist()
        if any(words[1:]):
            bad = [i for i, s in enumerate(self.slots) if any(s.index_errors().cpu().tolist())]
            raise RuntimeError(f"regnn_ns_hop: a transposed index build timed out waiting for its "
                               f"publish (sampler slots {bad}): those batches are incomplete")
        return int(words[0])
