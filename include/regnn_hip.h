/*
 * regnn_hip.h — C-ABI of libregnn_hip.so, the MI355X (gfx950) kernels behind RE-GNN's
 * relation-embedding message passing.
 *
 * The reference has no native code of its own: its hot path calls DGL 0.7.1's gspmm / gsddmm /
 * edge_softmax (full-batch layers) and torch_scatter / torch_sparse (ogbn-mag path) through their
 * Python APIs. Each entry point below names the reference call sites whose arithmetic it replaces.
 *
 * Conventions (all entry points)
 *  - Plain pointers + sizes; no framework types. Every buffer is device memory owned by the
 *    caller (PyTorch's caching allocator on the Python side); the library never allocates.
 *  - Work is enqueued on `stream` and is asynchronous; no host synchronisation, graph-capturable.
 *  - Return 0 on success, a REGNN_E* code otherwise (invalid argument / unsupported shape /
 *    launch failure). The Python wrapper raises RuntimeError on any non-zero return.
 *  - Graphs are compressed segments: CSR (segment = destination, idx = source) for forward
 *    aggregation, CSC (segment = source, idx = destination) for the transposed backward.
 *    `rel` holds 0-based relation ids (reference e_feat - 1, layer/REGraphConv.py:61) as uint8.
 *  - Feature rows are dense row-major [n, F]; dtype REGNN_F32 or REGNN_BF16 (storage type;
 *    accumulation is always fp32).
 *  - Segments with more than `split` edges are processed by the long-segment plan
 *    (long_ids/chunk_long/chunk_off, see regnn_spmm_fwd) so hubs do not serialise one wave;
 *    split == 0 disables splitting. Results are bitwise reproducible run to run: no float
 *    atomics (except regnn_ns_spmm_bwd, the sampled-block backward); cross-block reductions go
 *    through fixed-order slabs.
 */
#ifndef REGNN_HIP_H
#define REGNN_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;

enum { REGNN_OK = 0, REGNN_EINVAL = 1, REGNN_EUNSUPPORTED = 2, REGNN_ELAUNCH = 3 };
enum { REGNN_F32 = 0, REGNN_BF16 = 1 };
/* Flag or-ed into the dtype of the regnn_spmm_bwd* calls: the x rows passed are the rows the
 * forward gathered, out_scale * drop(x) (a producer that formed them, e.g. regnn_type_project),
 * not x itself; the per-edge relation dots then take them as they are and the node gradient is
 * <rows, gx_raw> / out_scale (out_scale > 0). Not combinable with edge_grad or the _next call. */
enum { REGNN_SELF_PRESCALED = 0x100 };

/* ABI version (bumped on any signature or semantics change; currently 46). */
int regnn_abi_version(void);

/* Tuning knob (process-wide, for A/B measurements; defaults are the shipped configuration).
 * key 1: grid cap of the grid-stride gather kernels (0 = resident capacity from the occupancy
 * API, the default; > 0 = fixed block count, at most 2048). key 2: rows gathered per lane per
 * step for 16-vector rows (F=64 fp32 / F=128 bf16): 0 = default (8), 4 or 16. key 3: fused
 * head variant (0 = next tile / next k-step operands prefetched, the default; 1 = plain).
 * key 4: rows in flight per lane group of regnn_row_scale (0 = default 1, 2 or 4).
 * Returns the previous value, -1 for an unknown key. */
int64_t regnn_tune(int32_t key, int64_t value);

/* Rows of the per-block relation-gradient slab that regnn_spmm_bwd / regnn_degree_bwd write
 * (one row of n_rel (x heads) floats per block); size the slab as rows * n_rel * heads floats. */
int64_t regnn_slab_rows(int64_t n_seg, int32_t n_chunk);

/* Long-segment relation counts: segments with more than `split` in-edges (long_ids[n_long]) are
 * not walked edge by edge in the degree kernels; long_cnt[l*n_rel + r] holds how many in-edges
 * of segment long_ids[l] carry relation r (a static property of the graph, built once).
 *
 * Weighted in-degree and its power norm.
 * Replaces: graph.update_all(fn.u_mul_e('nones','ew','m'), fn.sum('m','norm')) followed by
 *   th.pow(norm.clamp(min=1), power)   — layer/REGraphConv.py:66-75 (power -0.5),
 *   layer/REMixHopConv.py:58-64 (-0.5), layer/RESAGEConv.py:72-81 and REGINConv.py:162-166 (-1.0).
 * deg[v] = sum_{e in seg v} rel_table[rel[e]];  norm[v] = max(deg[v], 1)^power.
 * rel_table == NULL means weight 1 (unweighted in-count). */
int regnn_degree(const int32_t* ptr, const uint8_t* rel, const float* rel_table, int64_t n_seg,
                 float power, int32_t split, const int32_t* long_ids, int32_t n_long,
                 const int32_t* long_cnt, int32_t n_rel, float* deg, float* norm,
                 hipStream_t stream);

/* Backward of regnn_degree w.r.t. rel_table: slab[b][r] = partial over block b of
 *   sum_v g_norm[v] * power * max(deg,1)^(power-1) * [deg >= 1] * |{e in seg v : rel[e] = r}|.
 * Reduce the slab with regnn_rel_reduce. Requires n_rel <= 64. */
int regnn_degree_bwd(const int32_t* ptr, const uint8_t* rel, const float* deg, const float* g_norm,
                     int64_t n_seg, float power, int32_t n_rel, int32_t split,
                     const int32_t* long_ids, int32_t n_long, const int32_t* long_cnt,
                     float* slab, hipStream_t stream);

/* regnn_degree / regnn_degree_bwd from the graph's per-row relation histogram instead of its
 * relation ids: cnt [n_seg, n_rel] uint16 row-major, cnt[v, r] = number of in-edges of v with
 * relation r for the rows of at most `split` edges and 0 for the long rows (static per graph and
 * e_feat; RelPack.row_cnt builds it once). deg[v] = sum_r rel_table[r] cnt[v, r] (long rows from
 * long_cnt, as regnn_degree; ptr is read only for them), norm as regnn_degree. The backward
 * writes one slab row of n_rel partials per block (zero the slab, reduce with
 * regnn_rel_reduce). n_rel <= 16 (else REGNN_EINVAL: use the id-walking calls). */
int regnn_degree_cnt(const uint16_t* cnt, const float* rel_table, int32_t n_rel, int64_t n_seg,
                     float power, const int32_t* ptr, const int32_t* long_ids, int32_t n_long,
                     const int32_t* long_cnt, float* deg, float* norm, hipStream_t stream);
int regnn_degree_cnt_bwd(const uint16_t* cnt, const float* deg, const float* g_norm,
                         int64_t n_seg, float power, int32_t n_rel, const int32_t* long_ids,
                         int32_t n_long, const int32_t* long_cnt, float* slab,
                         hipStream_t stream);

/* Relation-embedding SpMM, forward direction.
 * Replaces DGL gspmm for graph.update_all(fn.u_mul_e('h','ew','m'), fn.sum('m','h'))
 *   (layer/REGraphConv.py:84-86, 91-93; with rel_table == NULL it is fn.copy_u,
 *   layer/REMixHopConv.py:80) and torch_scatter mean aggregation of PyG propagate
 *   (mag/regnn_layers.py:129,142-148, with out_scale = 1/in-count, bias = conv bias):
 *   y[i] = out_scale[i] * sum_{e in seg i} w(e) * in_scale[idx[e]] * x[idx[e]] + bias
 *   w(e) = (rel_table ? rel_table[rel[e]] : 1) * (edge_w ? edge_w[e] : 1)
 * Any of rel_table / edge_w / in_scale / out_scale / bias may be NULL.
 * Long-segment plan (all NULL / 0 when split == 0): long_ids[n_long] = segments with more than
 * `split` edges; chunk c covers edges [ptr[s] + k*chunk, ...) of s = long_ids[chunk_long[c]],
 * k = c - chunk_off[chunk_long[c]]. Chunk partial sums are combined by a fixed-order tree:
 * level k (k < n_levels) reduces partial rows [sb[p], sb[p+1]) (sb = level_sb + desc[k][0],
 * p < desc[k][1]) into row desc[k][2] + p; the last level leaves row desc[n-1][2] + l for long
 * segment l (n_levels == 0: row chunk_off[l]). level_desc is a HOST array [n_levels][3]
 * (int64: sb offset, n_out, output row base); chunk_partial is fp32 scratch
 * [n_chunk + sum n_out, F]. Deterministic for any chunk count (hub rows of 10^7 edges).
 * Scheduled form (split < 0, |split| is the threshold): chunk_long holds 2 * n_chunk entries and
 * chunk_long[n_chunk + i] is the chunk handled in processing slot i (a permutation; partial rows
 * and the tree are unchanged). The build orders slots by each chunk's first gathered row, so with
 * rows sorted by gathered id the chunks in flight share gathered rows in L2 / Infinity Cache.
 * Every entry point below that takes a plan accepts either form. */
int regnn_spmm_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                   const float* rel_table, const float* edge_w,
                   const float* in_scale, const float* out_scale, const float* bias,
                   const void* x, void* y, int64_t n_seg, int32_t F, int32_t dtype,
                   int32_t split, int32_t chunk, const int32_t* long_ids, int32_t n_long,
                   const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                   float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                   const int64_t* level_desc, hipStream_t stream);

/* regnn_spmm_fwd with a fused forward epilogue (the mag REGCNConv tail, forward only, e.g.
 * layer-wise inference, mag/regnn_ns.py:348-369):
 *   r = out_scale[i] * sum(...) + bias + (residual ? residual[i] : 0)
 *   (epi & 1) r = (r - mean(r)) / sqrt(var(r) + ln_eps) * ln_w + ln_b   (LayerNorm over the row,
 *             biased variance; ln_w / ln_b may be NULL; mag/regnn_layers.py:134-135)
 *   (epi & 2) r = max(r, 0)                                             (mag/regnn_ns.py:362)
 * residual rows have the dtype of y. */
int regnn_spmm_fwd_fused(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                         const float* rel_table, const float* edge_w,
                         const float* in_scale, const float* out_scale, const float* bias,
                         const void* x, void* y, int64_t n_seg, int32_t F, int32_t dtype,
                         int32_t split, int32_t chunk, const int32_t* long_ids, int32_t n_long,
                         const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                         float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                         const int64_t* level_desc, const void* residual, const float* ln_w,
                         const float* ln_b, float ln_eps, int32_t epi, hipStream_t stream);

/* regnn_spmm_fwd with a fused dropout of the gathered input rows. Replaces the nn.Dropout in
 * front of the aggregation (layer/REGraphConv.py:56 feat_dropout, and with it the model dropout
 * between layers, model/REGCN.py:43, when both precede the same aggregation): the rows are read
 * undropped and every gathered element is masked on the fly, so no dropped copy or mask tensor
 * is written. Mask spec (this build's; torch's Philox stream is not reproduced): per call a
 * 64-bit seed s read from device memory (*drop_seed, so a captured graph sees a new seed per
 * replay), key = fmix32(lo32(s) ^ fmix32(hi32(s) ^ 0x5BD1E995)) with fmix32 the murmur3
 * finaliser; element (row, f) lies in 16-byte vector v = f / EV (EV = 4 fp32, 8 bf16) of
 * nvec = F / EV; c = row * nvec + v; h_0 = fmix32(lo32(c) ^ key ^ rotl16(hi32(c))),
 * h_k = fmix32(h_{k-1} + 0x9E3779B9). 16-bit draws: feature f = v*EV + 2k + b keeps iff 16-bit
 * half b of h_k is < drop_keep16 (keep probability drop_keep16 / 65536). When drop_keep16 is a
 * multiple of 256 (p = 0.5, 0.25, ...), 8-bit draws: f = v*EV + 4k + b keeps iff byte b of h_k
 * is < drop_keep16 / 256 (same keep probability, half the hashing). Kept values are scaled by
 * drop_scale.
 * Rows must be 16 or 8 vectors (F = 64 fp32; 64 or 128 bf16), else REGNN_EUNSUPPORTED. */
int regnn_spmm_fwd_dropout(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                           const float* rel_table, const float* edge_w,
                           const float* in_scale, const float* out_scale, const float* bias,
                           const void* x, void* y, int64_t n_seg, int32_t F, int32_t dtype,
                           int32_t split, int32_t chunk, const int32_t* long_ids, int32_t n_long,
                           const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                           float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                           const int64_t* level_desc, const uint64_t* drop_seed,
                           uint32_t drop_keep16, float drop_scale, hipStream_t stream);

/* out[u][:] = (scale ? scale[u] : 1) * drop(x[u][:]) for n_rows rows of F features (dtype as
 * x; out may not alias x). drop is the regnn_spmm_fwd_dropout mask (same seed / threshold / scale,
 * same (row, vector) counter), or none when drop_seed is NULL. With z and dot (both or neither):
 * dot[u] = <x[u], z[u]> / scale[u] (fp32 accumulation).
 * Forward: the input pre-scale of layer/REGraphConv.py:73-76 (feat * norm) with the feat_dropout
 * of :56 in front of it, applied once per node so the aggregation gathers finished rows (no
 * per-edge mask hashing, no per-edge norm lookup); regnn_spmm_bwd_dropout with the same seed is
 * its backward. Backward: g * norm (post-scale side) with dot = <g, y> / norm, the output-side
 * term of d loss / d norm (layer/REGraphConv.py:97-98). */
int regnn_row_scale(const void* x, const float* scale, void* out, int64_t n_rows, int32_t F,
                    int32_t dtype, const uint64_t* drop_seed, uint32_t drop_keep16,
                    float drop_scale, const void* z, float* dot, hipStream_t stream);

/* Relation-embedding SpMM, fused backward over the transposed graph (CSC: segment = source u).
 * Replaces DGL GSpMM.backward (gspmm on the reverse graph + gsddmm 'dot' for the edge weight)
 * behind the same call sites as regnn_spmm_fwd, and the PyG/torch_scatter backward.
 *   gx[u]  = out_scale[u] * sum_{e: u->v} w(e) * in_scale[v] * g[v]          (transposed SpMM)
 *   slab   : per relation r, sum over edges with rel r of in_scale[v]*out_scale[u]*<g[v], x[u]>
 *            (d loss / d rel_table[r], SDDMM 'dot' fused; only when slab != NULL)
 *   edge_grad[e] (optional, this traversal's edge order): the same per-edge quantity
 *   node_grad[u] (optional) = <x[u], raw[u]> + (y ? <g[u], y[u]> / in_scale[u] : 0)
 *            with raw[u] = the sum above before out_scale: d loss / d norm[u] when
 *            in_scale == out_scale == norm (layer/REGraphConv.py:73-76,97-98).
 * x / y are the forward input / output rows (dtype as g). */
int regnn_spmm_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                   const float* rel_table, const float* edge_w,
                   const float* in_scale, const float* out_scale,
                   const void* g, const void* x, const void* y, void* gx,
                   float* slab, int32_t n_rel, float* edge_grad, float* node_grad,
                   int64_t n_seg, int32_t F, int32_t dtype,
                   int32_t split, int32_t chunk, const int32_t* long_ids, int32_t n_long,
                   const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                   float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                   const int64_t* level_desc, hipStream_t stream);

/* regnn_spmm_bwd through the fused dropout of regnn_spmm_fwd_dropout (same seed, threshold and
 * scale): x (the undropped forward input) is masked where the kernel reads it (relation bins,
 * edge and node gradients) and gx is the gradient w.r.t. the undropped rows (masked, scaled). */
int regnn_spmm_bwd_dropout(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                           const float* rel_table, const float* edge_w,
                           const float* in_scale, const float* out_scale,
                           const void* g, const void* x, const void* y, void* gx,
                           float* slab, int32_t n_rel, float* edge_grad, float* node_grad,
                           int64_t n_seg, int32_t F, int32_t dtype,
                           int32_t split, int32_t chunk, const int32_t* long_ids, int32_t n_long,
                           const int32_t* chunk_long, const int32_t* chunk_off, int32_t n_chunk,
                           float* chunk_partial, const int32_t* level_sb, int32_t n_levels,
                           const int64_t* level_desc, const uint64_t* drop_seed,
                           uint32_t drop_keep16, float drop_scale, hipStream_t stream);

/* regnn_spmm_fwd(_dropout when drop_seed != NULL) with the consumer's pre-scale folded into the
 * epilogue: when y is read by a next aggregation whose source rows are nx_scale * drop'(y)
 * (drop' = nx_seed / nx_keep16 / nx_dscale, the regnn_row_scale spec; nx_seed NULL = none),
 * this call writes them too, nx_out[v] = drop'(nx_scale[v] * y[v]) (dtype, from the stored y),
 * so the next aggregation gathers nx_out with no row pass (REGCN layer 0 -> layer 1,
 * layer/REGraphConv.py:56,73-76). */
int regnn_spmm_fwd_next(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                        const float* rel_table, const float* edge_w, const float* in_scale,
                        const float* out_scale, const float* bias, const void* x, void* y,
                        int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                        const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                        const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                        const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                        const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                        const float* nx_scale, const uint64_t* nx_seed, uint32_t nx_keep16,
                        float nx_dscale, void* nx_out, hipStream_t stream);

/* regnn_spmm_bwd(_dropout when drop_seed != NULL) with the producer's pre-scale folded into the
 * epilogue: when this op's input x is itself the output y' of an aggregation with post-scale
 * nx_scale (y' = nx_scale * A' x'), its backward needs nx_scale * g' and <g', y'> / nx_scale for
 * g' = gx (regnn_row_scale's backward pass). This call writes, besides gx,
 *   nx_out[u] = nx_scale[u] * gx[u]  (dtype),  nx_dot[u] = <gx[u], x[u]> / nx_scale[u]
 * (x undropped), so the producer's backward gathers nx_out directly: no separate row pass over
 * gx and x (REGCN layer 1 -> layer 0, layer/REGraphConv.py:73-76,97-98). */
int regnn_spmm_bwd_next(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                        const float* rel_table, const float* edge_w, const float* in_scale,
                        const float* out_scale, const void* g, const void* x, const void* y,
                        void* gx, float* slab, int32_t n_rel, float* edge_grad, float* node_grad,
                        int64_t n_seg, int32_t F, int32_t dtype, int32_t split, int32_t chunk,
                        const int32_t* long_ids, int32_t n_long, const int32_t* chunk_long,
                        const int32_t* chunk_off, int32_t n_chunk, float* chunk_partial,
                        const int32_t* level_sb, int32_t n_levels, const int64_t* level_desc,
                        const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                        const float* nx_scale, void* nx_out, float* nx_dot, hipStream_t stream);

/* out[k] = (accumulate ? out[k] : 0) + sum_{row < n_rows} slab[row][k], k < width, fixed order.
 * The slab is scratch: a wide one (width >= 4096, n_rows >= 256) is reduced in place in two
 * fixed-order stages (row splits, then the split sums), and its contents are clobbered. */
int regnn_rel_reduce(float* slab, int64_t n_rows, int32_t width, float* out,
                     int32_t accumulate, hipStream_t stream);

/* Long-segment plan of the GAT / per-head kernels below (the regnn_spmm_fwd split, as a struct):
 * segments with more than `split` edges (long_ids, n_long of them) are cut into chunks of `chunk`
 * edges (chunk c belongs to long segment chunk_long[c], the chunks of segment l are
 * [chunk_off[l], chunk_off[l+1])), processed by their own workgroups into fp32 partial rows
 * 0 .. n_chunk-1 of `partial` and combined per segment by the fixed-order tree of level_sb /
 * level_desc (HOST, [n_levels][3]: sb offset, n_out, row base; as regnn_spmm_fwd). partial holds
 * partial_rows rows of the width the entry point names; partial_floats is its capacity. A NULL
 * plan (or n_long = 0) runs every segment whole. The kernels skip long segments only when H is a
 * power of two <= 32 (their group forms); the generic forms run every segment whole. */
typedef struct regnn_seg_plan {
    int32_t split, chunk;
    const int32_t* long_ids; int32_t n_long;
    const int32_t* chunk_long; const int32_t* chunk_off; int32_t n_chunk;
    const int32_t* level_sb; int32_t n_levels; const int64_t* level_desc;
    int64_t partial_rows;
    float* partial; int64_t partial_floats;
} regnn_seg_plan;

/* GAT attention, forward. Replaces apply_edges(fn.u_add_v('el','er','e')) + ee add +
 * LeakyReLU + dgl edge_softmax (layer/REGATConv.py:80-88):
 *   s(e,h) = el[idx[e],h] + er[v,h] + (ee_table ? ee_table[rel[e]*H + h] : 0)
 *   z = leaky_relu(s, slope);  a(e,h) = exp(z - max_v z) / sum_v exp(z - max_v z)
 * over the in-edges of each destination v (CSR). a is written in CSR edge order [nnz, H]. */
int regnn_gat_softmax_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                          const float* ee_table, const float* el, const float* er,
                          int64_t n_seg, int32_t H, float slope, float* a,
                          const regnn_seg_plan* plan, hipStream_t stream);  /* partial width 2H */

/* GAT attention, backward (edge_softmax VJP + LeakyReLU + u_add_v), per destination v (CSR):
 *   gz = a * (ga - sum_v a*ga);  gs = gz * (s > 0 ? 1 : slope)
 *   gs_out[e,h] = gs (CSR order); ger[v,h] = sum_v gs;  slab: per (rel, h) sums of gs
 * (d loss / d ee_table) when slab != NULL (requires n_rel*H <= 256). */
int regnn_gat_softmax_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                          const float* ee_table, const float* el, const float* er,
                          const float* a, const float* ga, int64_t n_seg, int32_t H, float slope,
                          float* gs_out, float* ger, float* slab, int32_t n_rel,
                          const regnn_seg_plan* plan, hipStream_t stream);  /* partial width H */

/* Fused GAT forward (layer/REGATConv.py:80-92 in one pass: the u_add_v SDDMM + relation bias +
 * LeakyReLU, DGL edge_softmax over each destination's in-edges, and the per-head weighted SpMM):
 *   out[v,h,:] = sum_{e: u->v} softmax_v(e)[h] * x[u,h,:],  lse[v,h] = log sum_e exp(e[h])
 * with e[h] = LeakyReLU(el[u,h] + er[v,h] + ee_table[rel[e],h], slope), computed with an online
 * softmax (no [E, H] attention written). x / out [n, H*D] in dtype; lse [n_seg, H] fp32 (-inf for
 * a destination without in-edges, whose out row is 0). */
int regnn_gat_fused_fwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                        const float* ee_table, const float* el, const float* er, const void* x,
                        void* out, float* lse, int64_t n_seg, int32_t H, int32_t D, float slope,
                        int32_t dtype, const float* attn_l, const regnn_seg_plan* plan,
                        hipStream_t stream);  /* partial width H*D + 2H */
/* attn_l ([H, D] fp32, may be NULL): with fp32 rows, D % 4 == 0 and D / 4 a power of two the
 * kernel re-forms el[u] from the row it gathers (regnn_attn_dots_fwd's summation order, so
 * bitwise the el passed) instead of reading el: one random access per edge instead of two.
 * el must then be regnn_attn_dots_fwd(x, attn_l, ...)'s. */

/* The attention a[e,h] = exp(e[h] - lse[v,h]) (CSR edge order) of regnn_gat_fused_fwd, re-formed
 * for the backward. H a power of two <= 32. */
int regnn_gat_attn_lse(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                       const float* ee_table, const float* el, const float* er, const float* lse,
                       int64_t n_seg, int32_t H, float slope, float* a,
                       const regnn_seg_plan* plan, hipStream_t stream);  /* no partials */

/* Per-head weighted SpMM (GAT message passing, layer/REGATConv.py:90-91,
 * update_all(fn.u_mul_e('ft','a','m'), fn.sum('m','ft'))):
 *   y[v,h,:] = sum_{e in seg v} a[eid(e)*H + h] * x[idx[e],h,:],  eid(e) = perm ? perm[e] : e.
 * Rows are H*D wide, D % 4 == 0 (fp32). */
int regnn_spmm_heads_fwd(const int32_t* ptr, const int32_t* idx, const int32_t* perm,
                         const float* a, const void* x, void* y, int64_t n_seg, int32_t H,
                         int32_t D, int32_t dtype, const regnn_seg_plan* plan,
                         hipStream_t stream);  /* partial width H*D */

/* Fused backward of regnn_spmm_heads_fwd over the CSC (segment = source u, perm = CSC->CSR edge):
 *   gx[u,h,:] = sum_{e: u->v} a[perm[e],h] * g[v,h,:];   ga[perm[e],h] = <g[v,h,:], x[u,h,:]> */
int regnn_spmm_heads_bwd(const int32_t* ptr, const int32_t* idx, const int32_t* perm,
                         const float* a, const void* g, const void* x, void* gx, float* ga,
                         int64_t n_seg, int32_t H, int32_t D, int32_t dtype,
                         const regnn_seg_plan* plan, hipStream_t stream);  /* partial width H*D */

/* out[s,h] = sum_{e in seg s} vals[(perm ? perm[e] : e)*H + h]  (segment sum of edge values,
 * e.g. d loss / d el over the CSC). */
int regnn_segment_sum(const int32_t* ptr, const int32_t* perm, const float* vals, int64_t n_seg,
                      int32_t H, float* out, const regnn_seg_plan* plan,
                      hipStream_t stream);  /* partial width H */

/* Column sum of a row-major fp32 [rows, cols] matrix into per-block partial rows:
 * slab[b][c] = sum of column c over block b's row range (at most regnn_slab_rows()/2 blocks;
 * zero the slab first, then regnn_rel_reduce(slab, rows_of_slab, cols, out, 0)).
 * Replaces torch's grad.sum(0) for the bias gradient of nn.Linear heads over all nodes
 * (model/REGCN.py:32,45 out_lin), which ran far below HBM rate for N ~ 1e7 rows. */
int regnn_col_sum(const float* x, int64_t rows, int32_t cols, float* slab, hipStream_t stream);

/* Per-type input projection fused with the first aggregation's pre-scale (model/REGCN.py:31-35
 * fc_list, then layer/REGraphConv.py:56,73-76 feat_dropout and feat * norm): for the rows of one
 * node type, x [rows, K] (dtype), W [F, K] fp32, b [F] fp32 (16-byte aligned):
 *   h [row0 + r]  = x[r] W^T + b                          (rows of the concatenated layer input)
 *   xs[row0 + r] = scale[row0 + r] * drop(h[row0 + r])     (as regnn_row_scale(h), same mask)
 * h / xs: dtype, [*, F] row-major. fp32-accurate (bf16x6 MFMA). F must be 64; K <= 256
 * (REGNN_EUNSUPPORTED above: use a GEMM + regnn_row_scale). scale may be NULL (1). h may be
 * NULL: only xs is written (its consumer's backward then takes xs, REGNN_SELF_PRESCALED). */
int regnn_type_project(const void* x, int64_t rows, int32_t K, int32_t F, int32_t dtype,
                       const float* W, const float* b, const float* scale,
                       const uint64_t* drop_seed, uint32_t drop_keep16, float drop_scale,
                       int64_t row0, void* h, void* xs, hipStream_t stream);

/* Weight and bias gradient of a Linear(K -> C) layer over n rows (model/REGCN.py:31-35 fc_list
 * backward): per-block partial slab rows [64*K + 64] (fp32): columns [0, 64*K) hold
 * (g^T x)[c][k] at c*K + k (d weight, rows c >= C zero), columns [64*K, +64) the column sums of g
 * (d bias). g [n, C] with row stride ldg (bf16: rows 8-byte aligned), x [n, K] row-major
 * 16-byte aligned, both dtype; fp32-accurate bf16x6 MFMA, one pass over g and x per 64-feature block.
 * C <= 64, K in {64, 128, 256} (else REGNN_EUNSUPPORTED). At most slab_rows (>= 8) rows are
 * written: zero the slab first, reduce with regnn_rel_reduce. */
int regnn_linear_wgrad(const void* g, int64_t n, int32_t C, int64_t ldg, const void* x,
                       int32_t K, int32_t dtype, float* slab, int32_t slab_rows,
                       hipStream_t stream);

/* Row-wise softmax cross-entropy of the output head over `rows` logit rows (stride ld):
 * loss_rows[r] = logsumexp(z_r) - z_r[labels[r]];  p[r, c] = scale * (softmax(z_r)_c - [c == y_r])
 * (p dense [rows, cols]); the CE of run_regnn.py:147 and its gradient in one pass. */
int regnn_softmax_xent(const float* logits, int64_t rows, int32_t cols, int64_t ld,
                       const int64_t* labels, float scale, float* p, float* loss_rows,
                       hipStream_t stream);

/* Fused output head (run_regnn.py:146-148: out_lin over all nodes, log_softmax + nll over the
 * train rows): logits[rows, C] = h[rows, K] W[C, K]^T + b  (b may be NULL), and for the first
 * n_loss rows loss_rows / p exactly as regnn_softmax_xent. logits and p have row stride ld >= C
 * (ld = 16 * ceil(C / 16) puts every row on 64-byte boundaries: the L2 then merges each row's
 * stores into whole lines). fp32-accurate MFMA (bf16x6 split for C <= 368, f32 MFMA above);
 * K must be 64 and C <= 384 (else REGNN_EINVAL: use a GEMM + regnn_softmax_xent); h 16-byte
 * aligned. */
int regnn_head_fwd(const float* h, int64_t rows, int32_t K, const float* W, const float* b,
                   int32_t C, int64_t ld, const int64_t* labels, int64_t n_loss, float scale,
                   float* logits, float* p, float* loss_rows, hipStream_t stream);

/* Backward of the fused output head from its softmax gradient p [n, C] with row stride ld
 * (regnn_head_fwd), each part reading p once (fp32-accurate bf16x6 MFMA):
 *   gh (optional, [n_out, K], n_out >= n, 16-byte aligned) = gscale[0] * p W on rows < n
 *      (gscale NULL: 1) and 0 on rows [n, n_out) (nodes without a loss term)
 *   slab (optional): per-block partial rows [rows_used, Cp*K + Cp], Cp = 16 * ceil(C/16):
 *     columns [0, Cp*K) hold (p^T h)[c][k] at c*K + k (d out_lin.weight), columns [Cp*K, +Cp)
 *     the column sums of p (d out_lin.bias). At most slab_rows rows are written: zero the slab
 *     first and reduce its slab_rows rows with regnn_rel_reduce (fixed order).
 *     K must be 64, C <= 384. */
int regnn_head_bwd(const float* p, int64_t n, int32_t C, int64_t ld, int32_t K, const float* W,
                   const float* h, const float* gscale, float* gh, int64_t n_out, float* slab,
                   int32_t slab_rows, hipStream_t stream);

/* regnn_head_fwd without the p output: the same logits, and loss_lse [2, n_loss] holds the loss
 * rows (row 0) and each loss row's log-sum-exp (row 1), from which regnn_head_bwd_z re-forms
 * p = scale * (exp(z - lse) - [c == y]) out of the logits rows it already has. The forward then
 * stores n_loss x ld fp32 fewer (10.4 GB at mag-10x). Same shape limits as regnn_head_fwd. h rows
 * in dtype: REGNN_F32, or REGNN_BF16 (a bf16 feature pipeline's rows, read as they are: exact in
 * the first bf16x6 split; C <= 368, else REGNN_EUNSUPPORTED). */
int regnn_head_fwd_lse(const void* h, int64_t rows, int32_t K, const float* W, const float* b,
                       int32_t C, int64_t ld, const int64_t* labels, int64_t n_loss,
                       float* logits, float* loss_lse, int32_t dtype, hipStream_t stream);

/* regnn_head_bwd / regnn_head_gh_next from the logits rows z [n, C] (row stride ld) of
 * regnn_head_fwd_lse instead of a stored p: p[r, c] = scale * (exp(z[r, c] - lse[r]) - [c ==
 * labels[r]]) is formed on the fly inside the gh and slab kernels (bf16x6 MFMA). gh, slab and
 * (nx_scale, nx_out, nx_dot) have the meaning of those calls; h ([n, K] in dtype) feeds the
 * slab (p^T h), hx (the head input as the aggregation stored it, dtype) the nx dot. gh, hx and nx_out
 * are stored in dtype (REGNN_F32: 16-byte aligned rows; REGNN_BF16: 8-byte aligned, gh rounded
 * first and nx_out = round(nx_scale * gh) from the rounded gh, as a stored bf16 gradient would
 * be). Either part (gh / slab) may be NULL. */
int regnn_head_bwd_z(const float* z, int64_t n, int32_t C, int64_t ld, int32_t K,
                     const float* W, const void* h, const float* gscale, void* gh,
                     int64_t n_out, float* slab, int32_t slab_rows, const float* lse,
                     const int64_t* labels, float scale, const void* hx, const float* nx_scale,
                     void* nx_out, float* nx_dot, int32_t dtype, hipStream_t stream);

/* regnn_head_bwd's gh (gscale * p W, rows [n, n_out) zero) with the consumer-side row pass of
 * h's producer folded in: when h is the output of an aggregation with post-scale nx_scale, its
 * backward needs nx_scale * gh and <gh, h> / nx_scale; this call writes, besides gh,
 *   nx_out[u] = nx_scale[u] * gh[u],  nx_dot[u] = <gh[u], h[u]> / nx_scale[u]
 * (nx_dot zero for the rows without a loss term, whose h is not read; nx_out rows [n, n_out) are
 * NOT written: the gradient there is zero, and the consumer gathers only edges into rows < n). K = 64, fp32, 16-byte aligned
 * gh / h / nx_out (REGCN's last layer -> out_lin, run_regnn.py:146-148). */
int regnn_head_gh_next(const float* p, int64_t n, int32_t C, int64_t ld, int32_t K,
                       const float* W, const float* gscale, float* gh, int64_t n_out,
                       const float* nx_scale, const float* h, float* nx_out, float* nx_dot,
                       hipStream_t stream);

/* Inference head (mag/regnn_ns.py:367 out_lin over every node, then the caller's argmax,
 * regnn_ns.py:379): out[r] = argmax_c (h[r] W^T + b)[c] (first maximal class, as torch.argmax),
 * fp32 MFMA as regnn_head_fwd, without writing the [rows, C] logits. K must be 64, C <= 384. */
int regnn_head_argmax(const float* h, int64_t rows, int32_t K, const float* W, const float* b,
                      int32_t C, int64_t* out, hipStream_t stream);

/* GAT attention logits (layer/REGATConv.py:68-69 el = (ft * attn_l).sum(-1), er likewise):
 * ft [N, H, D], attn_l / attn_r [H, D] -> el, er [N, H]. */
int regnn_attn_dots_fwd(const float* ft, const float* attn_l, const float* attn_r, int64_t N,
                        int32_t H, int32_t D, float* el, float* er, hipStream_t stream);

/* Backward of regnn_attn_dots_fwd: gft[n,h,:] = gel[n,h] attn_l[h,:] + ger[n,h] attn_r[h,:]
 * (written, not accumulated), and slab [slab_rows, 2*H*D] of per-block partial sums whose
 * column sums (regnn_rel_reduce, width 2*H*D) are [d attn_l | d attn_r]. Every row is written. */
int regnn_attn_dots_bwd(const float* ft, const float* attn_l, const float* attn_r,
                        const float* gel, const float* ger, int64_t N, int32_t H, int32_t D,
                        float* gft, float* slab, int32_t slab_rows, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * GATv2 scores and the edge softmax over per-edge logits (re_gatv2.hip; H a power of two <= 32
 * for the softmax entry points; D % 4 == 0 with D / 4 a power of two for the score kernels).
 * plan (may be NULL; ABI 41): the CSR's (CSC's for bwd_src) long-segment plan, as REGATConv's
 * entry points take it: hub rows run as chunks on groups of their own, their segment sums /
 * max / dot combined by the plan's fixed-order tree. Partial widths: score_fwd 0,
 * score_bwd_dst / _src H*D, edge_softmax_fwd 2H, edge_softmax_bwd H.
 * --------------------------------------------------------------------------------------- */

/* GATv2 score SDDMM (layer/REGATv2Conv.py:139-141; mag/regnn_layers.py:399-403), CSR order:
 *   s[e,h] = sum_d att[h*D+d] * LeakyReLU(fs[idx[e], h*D+d] + fd[v, h*D+d], slope). */
int regnn_gatv2_score_fwd(const int32_t* ptr, const int32_t* idx, const float* fs, const float* fd,
                          const float* att, int64_t n_seg, int32_t H, int32_t D, float slope,
                          float* s, const regnn_seg_plan* plan, hipStream_t stream);

/* Its backward, destination side (CSR): gfd[v] = sum_{e in seg v} gs[e,h] * att * lrelu'(pre),
 * and per-block partials of d att = sum_e gs[e,h] * LeakyReLU(pre) in att_slab
 * [slab_rows, H*D] (zero-filled by the caller; the launches write rows < slab_rows: with a
 * plan's chunks the per-segment pass takes rows < slab_rows / 2, the chunk pass the rest;
 * reduce every row with regnn_rel_reduce). */
int regnn_gatv2_score_bwd_dst(const int32_t* ptr, const int32_t* idx, const float* fs,
                              const float* fd, const float* att, const float* gs, int64_t n_seg,
                              int32_t H, int32_t D, float slope, float* gfd, float* att_slab,
                              int32_t slab_rows, const regnn_seg_plan* plan, hipStream_t stream);

/* Its backward, source side (CSC, csc2csr maps a CSC position to the CSR edge position of gs):
 *   gfs[u] = sum_{e: u->v} gs[e,h] * att * lrelu'(fs[u] + fd[v]). */
int regnn_gatv2_score_bwd_src(const int32_t* csc_ptr, const int32_t* csc_idx,
                              const int32_t* csc2csr, const float* fs, const float* fd,
                              const float* att, const float* gs, int64_t n_src, int32_t H,
                              int32_t D, float slope, float* gfs, const regnn_seg_plan* plan,
                              hipStream_t stream);

/* Edge softmax over per-edge logits z = s[e,h] + (ee_table ? ee_table[rel[e]*H + h] : 0), per
 * destination (CSR):
 *   gmax == NULL: a = exp(z - max_v z) / sum_v exp(z - max_v z)     (dgl edge_softmax,
 *                 layer/REGATv2Conv.py:152)
 *   gmax != NULL: a = exp(z - *gmax) / (sum_v exp(z - *gmax) + eps)  (mag/utils.py:45-57 with
 *                 the global max read from device memory: far-below-max segments underflow to 0
 *                 exactly as the reference's). */
int regnn_edge_softmax_fwd(const int32_t* ptr, const float* s, const uint8_t* rel,
                           const float* ee_table, const float* gmax, float eps, int64_t n_seg,
                           int32_t H, float* a, const regnn_seg_plan* plan, hipStream_t stream);

/* Backward (both forms; the global max's own gradient is exactly 0 up to the eps term):
 *   gz = a * (ga - sum_v a*ga) (CSR order); slab (optional, regnn_slab_rows() rows): per-block
 *   (rel, h) sums of gz. */
int regnn_edge_softmax_bwd(const int32_t* ptr, const uint8_t* rel, const float* a,
                           const float* ga, int64_t n_seg, int32_t H, float* gz, float* slab,
                           int32_t n_rel, const regnn_seg_plan* plan, hipStream_t stream);

/* GAT v1 scores written per edge (CSR): s = LeakyReLU(el[idx[e],h] + er[v,h] + ee[rel[e],h]),
 * for the global max of the ogbn-mag softmax (mag/regnn_layers.py:297-307). */
int regnn_gat_scores(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                     const float* ee_table, const float* el, const float* er, int64_t n_seg,
                     int32_t H, float slope, float* s, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Neighbour sampler (replaces torch_sparse SparseTensor.sample_adj behind PyG NeighborSampler,
 * mag/regnn_ns.py:206-214). Spec (this build's, documented in DESIGN.md; torch_sparse's RNG is
 * not reproducible): for target t with in-degree d and fan-out k (k < 0: all):
 *   d <= k or k < 0  -> all in-edges in CSR order;
 *   else Floyd sampling of k distinct positions in [0,d) drawing
 *        r_j = regnn_hash(seed, t_global, j) for j = d-k .. d-1, pos = (r_j * (j+1)) >> 32,
 *   output in ascending position order.
 * --------------------------------------------------------------------------------------- */

/* counts[i] = min(deg(targets[i]), k) (or deg when k < 0). */
int regnn_sample_count(const int32_t* ptr, const int32_t* targets, int64_t n_targets, int32_t k,
                       int32_t* counts, hipStream_t stream);

/* Fill sampled neighbours: out_src[offs[i] + q] = global source id, out_eid[...] = CSR edge id.
 * offs = exclusive prefix sum of counts (n_targets + 1 entries). Requires k <= 64. */
int regnn_sample_fill(const int32_t* ptr, const int32_t* idx, const int32_t* targets,
                      int64_t n_targets, int32_t k, uint64_t seed, const int32_t* offs,
                      int32_t* out_src, int32_t* out_eid, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Device-resident neighbour-sampled step (re_ns.hip). The same sampler spec as above, with no
 * host sizes anywhere, so a whole mag/regnn_ns.py training step (sample, fwd, bwd, Adam) runs
 * without a host synchronisation and can be captured in a HIP graph.
 *
 *  state  int64 [8] (device): [0] base seed, [1] epoch, [2] step within the epoch (this rank),
 *         [3] global batch of the current step (the hop seeds use it), [4] step stamp (dedup
 *         tables), [5] running count of aggregated edges (every hop's block incl. self loops).
 *         Zero it once (then set [0], [1]); regnn_ns_batch advances [2]-[4] per step.
 *  sizes  int32 [16] (device): [h] = |n_id| after h hops ([0] = batch size), [8 + h] = edges of
 *         hop h's block (sampled + one self loop per target).
 *  n_id   int32 [cap_src]: hop h's targets n_id[0, sizes[h]), it appends its new sources in
 *         first-seen order (the sampler_oracle / PyG n_id contract).
 *  g2l, first  uint64 [num_nodes] dedup tables: g2l zero-filled, first all-ones, once.
 *  Per-hop scratch (cap_dst = capacity of the hop's targets, k = fan-out, cap_e = cap_dst*(k+1)):
 *  samp, spos [cap_dst*k] int32; scnt [cap_dst] int32; gsrc [cap_e] int32; flag [cap_e] uint8;
 *  tiles [ceil(cap_e/1024) + 4] int32, zero-filled once; status [ceil(cap_dst/1024)] uint64
 *  (row-offset look-back, zero-filled once).
 *  Block output (mag/regnn_layers.py:90-99 with self_loop_type 2): blk_ptr [cap_dst+1],
 *  blk_idx [cap_e] (local source ids; row i's self loop last), blk_rel [cap_e] uint8 (edge type
 *  etype[csr position], or num_edge_types + ntype[target] for the loop), blk_pos [cap_e] (CSR
 *  position of the sampled edge in the global graph, -1 for the loop), blk_row [cap_e] (the
 *  target row of each edge: the transposed pass of the fused step walks edges, not rows),
 *  inv [cap_dst] = 1 / (sampled + 1) (torch_scatter 'mean', mag/regnn_layers.py:37). Rows >=
 *  sizes[hop] empty.
 * --------------------------------------------------------------------------------------- */

/* Step prologue: rank r of `world` takes global batch g = (r + state[2] * world) mod nb of the
 * epoch permutation perm [n_perm] (nb = ceil(n_perm / batch); every rank runs the same number of
 * steps, a rank past the end wraps), writes its targets to n_id[0, cnt) and sizes[0] = cnt,
 * state[3] = g, and advances state[2] and the dedup stamp state[4] (by one, or, with stamp_src
 * non-null, to ++*stamp_src: one int64 counter shared by samplers that use the same dedup
 * tables one after another, so their stamps stay increasing). */
/* The wide NS model's small per-step ops, one launch each (ABI 42):
 * regnn_ns_labels: y[i] = labels[n_id[i]] for i < sizes[0] (the batch's live targets), else
 *   `ignore` (nll_loss's ignore_index), i < B -- replaces mag/regnn_ns.py:404's y gather plus the
 *   mask of a capacity-sized batch;
 * regnn_rel_tab: out = leaky_relu(alpha rw, slope) (gtab NULL; mag/regnn_layers.py:110-111) or,
 *   with gtab, its backward out = d rw = gtab alpha (alpha rw > 0 ? 1 : slope), n entries. */
int regnn_ns_labels(const int32_t* n_id, const int32_t* sizes, const int64_t* labels, int32_t B,
                    int64_t ignore, int64_t* y, hipStream_t stream);
/* log_softmax + nll_loss over B rows of C fp32 logits z (row-major), labels y (`ignore` rows
 * skipped): forward (a wave per row, then a fixed-order sum: deterministic) writes lse[B], the
 * scratch rowloss[2 B] and out[2] = {mean loss over the valid rows, their count}; backward gz =
 * g[0] / out[1] * (softmax(z) - onehot(y)), zero rows for ignored labels (ABI 42;
 * mag/regnn_ns.py:404-405's log_softmax / nll pair). */
int regnn_softmax_xent_fwd(const float* z, const int64_t* y, int32_t B, int32_t C, int64_t ignore,
                           float* lse, float* rowloss, float* out, hipStream_t stream);
int regnn_softmax_xent_bwd(const float* z, const int64_t* y, const float* lse, const float* stat,
                           const float* g, int32_t B, int32_t C, int64_t ignore, float* gz,
                           hipStream_t stream);
/* The same loss for a capacity-sized sampled batch in one launch (ABI 45): y[i] = labels[n_id[i]]
 * for i < sizes[0], else `ignore` (written to y[B], as regnn_ns_labels), lse / rowloss as
 * regnn_softmax_xent_fwd, and out[2] from the last workgroup to finish (ticket: one int32, zero
 * on entry and on return; rows summed in a fixed order). regnn_xent_bwd_colsum: gz as
 * regnn_softmax_xent_bwd, plus gb[c] = sum over rows of gz[r][c] (fixed order) -- out_lin's bias
 * gradient (mag/regnn_ns.py:346 out_lin + :404-405 log_softmax / nll) without a reduction of
 * its own. */
int regnn_ns_xent_fwd(const float* z, const int32_t* n_id, const int32_t* sizes,
                      const int64_t* labels, int32_t B, int32_t C, int64_t ignore, int64_t* y,
                      float* lse, float* rowloss, float* out, int32_t* ticket, hipStream_t stream);
int regnn_xent_bwd_colsum(const float* z, const int64_t* y, const float* lse, const float* stat,
                          const float* g, int32_t B, int32_t C, int64_t ignore, float* gz,
                          float* gb, hipStream_t stream);
int regnn_rel_tab(const float* rw, const float* gtab, int32_t n, float alpha, float slope,
                  float* out, hipStream_t stream);
/* regnn_rel_tab over `count` <= 4 tables (rw[t] of n[t] entries; gtab NULL: forward, else every
 * gtab[t] set: backward) in one launch: every conv layer's relation table at once. */
int regnn_rel_tabs(const float* const* rw, const float* const* gtab, float* const* out,
                   const int32_t* n, int32_t count, float alpha, float slope, hipStream_t stream);

int regnn_ns_batch(const int64_t* perm, int64_t n_perm, int32_t batch, int32_t rank,
                   int32_t world, int64_t* state, int32_t* n_id, int32_t* sizes,
                   int64_t* stamp_src, hipStream_t stream);

/* One sampling hop (replaces torch_sparse sample_adj for one layer of PyG NeighborSampler,
 * mag/regnn_ns.py:206-214): targets n_id[0, sizes[hop]) of the global CSR (ptr, idx; etype =
 * 0-based edge type per CSR position, ntype = node type per node), fan-out k in [1, 64], seed
 * hop_seed(state[0], state[1], state[3], hop). Writes the block (above), appends the new nodes,
 * sets sizes[hop + 1] and sizes[8 + hop], adds the block's edges to state[5]. Optional (all
 * three or none): with local = the per-node row in its type's table (mag local_node_idx), also
 * writes each block edge's source node type edge_type [cap_e] int32 and table row edge_off
 * [cap_e] int64 (what the fused step's layer 0 gathers by). meta_only (needs the three): the
 * hop whose sources only feed layer 0 by (type, row) — no first-seen de-duplication, no n_id
 * append (sizes[hop + 1] = sizes[hop]), blk_idx of the sampled edges not written; blk_ptr,
 * blk_rel, blk_pos, inv, the self loops and the edge meta as above (3 launches instead of 6).
 * Optional (all four or none, not with meta_only): the block's transposed index -- csc_cnt
 * [cap_e] (scratch), csc_ptr [cap_e + 1] (source i's edges are csc_ent[csc_ptr[i] ..
 * csc_ptr[i + 1]) over the n_{hop+1} sources), csc_ent [cap_e] = target row << 8 | relation
 * (the order inside a segment is unspecified), csc_long [REGNN_CSC_LONG_INTS] = the number of
 * sources with more than 16 edges (hub rows), then their ids ascending; at
 * [REGNN_CSC_LONG_NPIECE] the number of hub pieces and from [REGNN_CSC_LONG_TAB] one int4 per
 * piece (source, first entry in csc_ent, entries <= REGNN_CSC_PIECE, li << 16 | piece index
 * << 8 | pieces of the row), a row's pieces consecutive (one more launch; cap_e <= 32768).
 * strided = 1: the block in the fixed-stride layout instead of the CSR -- row i's edges at
 * [i S, i S + cnt_i) (S = k + 1, cnt_i = scnt[i], sampled positions ascending), its self loop at
 * i S + cnt_i, the other slots empty (blk_idx -1); blk_ptr is not written. Sampling and
 * placement run as one launch (no row-offset scan), the de-duplication as one pass (decoupled
 * look-back over status), the transposed index by many blocks in one launch (the last block
 * to resolve scans the counts and publishes csc_ptr, then every block places its entries):
 * 3 launches with de-duplication and the transposed index, 1 meta-only. Strided buffer sizes:
 * tiles >= ceil(cap_e / 1024) + 4 ints (the CSR path's tile words, then the index's own arrival
 * ticket, published stamp and sticky error word at tiles[ceil(cap_e / 1024) + 3]: 1 when a block
 * gave up waiting for the publish and placed nothing -- the caller checks it), status >=
 * ceil(cap_e / 1024) int64 (ABI 43). sizes[8 + hop] must be zero on entry (regnn_ns_batch zeroes sizes[8 ..]);
 * the hop adds its edges to it and to state[5]. strided = 2 (with the transposed index, no
 * edge meta): everything but the transposed index and the sampled edges' blk_idx, which a
 * second call with strided = 3 and the same arguments then writes (on another stream if the
 * caller wants: nothing the next hop reads depends on it). */
#define REGNN_CSC_PIECE 1024
#define REGNN_CSC_LONG_CAP (32768 / 17 + 1)          /* hub rows of a <= 32768-edge block */
#define REGNN_CSC_LONG_NPIECE (REGNN_CSC_LONG_CAP + 1)
#define REGNN_CSC_LONG_TAB (((REGNN_CSC_LONG_NPIECE + 1) + 3) / 4 * 4)
#define REGNN_CSC_LONG_MAXPIECE (32768 / REGNN_CSC_PIECE + REGNN_CSC_LONG_CAP)
#define REGNN_CSC_LONG_INTS (REGNN_CSC_LONG_TAB + 4 * REGNN_CSC_LONG_MAXPIECE)
int regnn_ns_hop(const int32_t* ptr, const int32_t* idx, const uint8_t* etype,
                 const int32_t* ntype, int32_t num_edge_types, int32_t k, int32_t hop,
                 int64_t* state, int32_t* sizes, int32_t* n_id, int32_t cap_dst,
                 uint64_t* g2l, uint64_t* first, int32_t* samp, int32_t* spos, int32_t* scnt,
                 int32_t* gsrc, uint8_t* flag, int32_t* tiles, uint64_t* status,
                 int32_t* blk_ptr, int32_t* blk_idx, uint8_t* blk_rel, int32_t* blk_pos,
                 int32_t* blk_row, float* inv, const int64_t* local, int32_t* edge_type,
                 int64_t* edge_off, int32_t meta_only, int32_t* csc_cnt, int32_t* csc_ptr,
                 int32_t* csc_ent, int32_t* csc_long, int32_t strided, hipStream_t stream);

/* The fused step's outer (meta-only, strided) hop with layer 0's parameter-free input sums
 * (relation slots: each (target type, source type) pair has one relation). Samples hop `hop` as
 * regnn_ns_hop(meta_only = 1, strided = 1) does -- the same slots, scnt, inv, blk_rel, edge_type /
 * edge_off, sizes[hop + 1] = sizes[hop], edge counts into sizes[8 + hop] and state[5] -- and then
 * sums each row i's sampled raw input rows (tables[t] rows local[u], K = 128 fp32) per source node
 * type: s_agg[i][t][:] = sum of the rows of type t (unweighted), s_w[i][t] = their count,
 * u_self[i][:] = the self loop's row, u_rel[i][t] = the relation of type t's edges (-1: none),
 * u_rel[i][T] = the self loop's relation (regnn_nsm_work's layer-0 buffers, read by
 * regnn_nsm_step with pre_sums = 1; they depend on the batch only, so the sampler computes them
 * ahead of the model). T = n_types in [1, 4], k <= 63, tables / s_agg / u_self 16-byte aligned.
 * One launch. The summation order is fixed (the result is a function of the batch).
 * csc (may be NULL; ABI 42): an earlier hop's transposed index, whose regnn_ns_hop call ran with
 * strided = 2 (de-duplication done, index left out), built by extra workgroups of the same launch
 * (regnn_ns_hop strided = 3's work, beside the sums instead of before them; same state / sizes). */
typedef struct regnn_ns_csc_job {
    int32_t hop;                /* that hop */
    int32_t cap_e;              /* its block's slots: cap_dst * (k + 1) <= 32768 */
    const int32_t* gsrc;        /* its buffers, as passed to regnn_ns_hop */
    const uint64_t* g2l;
    int32_t* blk_idx;
    const int32_t* blk_row;
    const uint8_t* blk_rel;
    int32_t* csc_cnt;
    int32_t* tiles;             /* >= ceil(cap_e / 1024) + 4 ints (as regnn_ns_hop) */
    int32_t* csc_ptr;
    int32_t* csc_ent;
    int32_t* csc_long;
} regnn_ns_csc_job;
int regnn_ns_hop_typed_sums(const int32_t* ptr, const int32_t* idx, const uint8_t* etype,
                            const int32_t* ntype, int32_t num_edge_types, int32_t k, int32_t hop,
                            int64_t* state, int32_t* sizes, const int32_t* n_id, int32_t cap_dst,
                            int32_t* scnt, uint8_t* blk_rel, float* inv, const int64_t* local,
                            int32_t* edge_type, int64_t* edge_off, const float* const* tables,
                            int32_t n_types, int32_t K, float* s_agg, float* s_w, float* u_self,
                            int32_t* u_rel, const regnn_ns_csc_job* csc, hipStream_t stream);

/* Backward of a sampled block's aggregation y[v] = out_scale[v] sum_e rel_table[rel_e] x[idx_e]
 * (+ bias) over rows v < n_rows (the forward is regnn_spmm_fwd on the block):
 *   gx[idx_e] += rel_table[rel_e] * out_scale[v] * g[v]   (gx zero-filled by the caller; hardware
 *                                                          float atomics: a block has no CSC)
 *   slab[b][r] (optional) = block b's partial of sum_{e: rel_e = r} out_scale[v] <g[v], x[idx_e]>
 *   (reduce with regnn_rel_reduce over min(n_rows, 2048) rows; zero it first).
 * fp32 rows, F % 4 == 0. The atomics make the summation order run-dependent (the reference's
 * torch_scatter CUDA backward is the same); every other entry point stays deterministic. */
int regnn_ns_spmm_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                      const float* rel_table, const float* out_scale, const float* g,
                      const float* x, float* gx, float* slab, int32_t n_rel, int64_t n_rows,
                      int32_t F, hipStream_t stream);

/* regnn_ns_spmm_bwd as a gather over the block's transposed index (regnn_ns_hop csc_ptr /
 * csc_ent: per local source u its entries (target row v << 8 | relation r)):
 *   gx[u] = sum_{entries of u} rel_table[r] out_scale[v] g[v]      (every row u < cap_rows
 *           written once; rows u >= sizes[size_idx] (the batch's sources) get zeros)
 *   slab[b][r] (optional) = block b's partial of sum out_scale[v] <g[v], x[u]> over relation r
 *   (launches slab_rows blocks; reduce with regnn_rel_reduce; LDS bins per row group, added in
 *   entry order and summed in group order: bitwise reproducible).
 * sizes may be null (then every row < cap_rows is live). F in {64, 128, 256, 512, 1024, 2048}.
 * hub_work (optional, regnn_ns_csc_hub_work_floats(F) floats): the hub rows (csc_long's piece
 * table) are cut into chunks of (256 / min(64, F / 4)) * 8 entries, one workgroup each, and
 * their sums added per row in chunk order by a second launch (without: a workgroup per hub row). */
int64_t regnn_ns_csc_hub_work_floats(int32_t F);
int regnn_ns_spmm_bwd_csc(const int32_t* csc_ptr, const int32_t* csc_ent, const int32_t* csc_long,
                          const float* rel_table, const float* out_scale, const float* g,
                          const float* x, float* gx, float* slab, int32_t n_rel,
                          const int32_t* sizes, int32_t size_idx, int64_t cap_rows, int32_t F,
                          int32_t slab_rows, float* hub_work, hipStream_t stream);

/* Typed aggregation of raw input rows over a sampled block (layer 0 of the NS REGNN at any hidden
 * width; mag/regnn_ns.py:300-326 group_input + mag/regnn_layers.py:101-148, replacing the
 * reference's per-type Linear over every sampled node and x_src @ W before propagate):
 *   S[v][t][:] = sum_{e in row v, ntype[n_id[idx_e]] = t} rel_table[rel_e] tables[t][local[n_id[idx_e]]][:]
 *   wsum[v][t] = sum over the same edges of rel_table[rel_e]
 * for v < n_rows (rows with ptr[v] == ptr[v + 1] get zeros). With e_type / e_off (a meta-only
 * hop's per-edge source node type and table row, regnn_ns_hop) the edge's type and row are read
 * from them and idx / n_id / ntype / local may be null. The caller projects
 * a = inv (S W_c + wsum b_c) + bias with W_c[t] = W_t^T W_0, b_c[t] = b_t W_0 (linearity).
 * K in {64, 128} fp32 (rows 16-byte aligned), 1 <= n_types <= 8, tables[t] non-null. Row
 * strides: S row v at S + v ld_s (ld_s >= n_types K, a multiple of 4, S 16-byte aligned), wsum row v
 * at wsum + v ld_w (ld_w >= n_types): the caller can place wsum as S's last n_types columns
 * (one [n][T K + T] operand, so the projection is one GEMM against [W_c; b_c]). */
int regnn_ns_typed_agg(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                       const float* rel_table, const int32_t* n_id, const int32_t* ntype,
                       const int64_t* local, const int32_t* e_type, const int64_t* e_off,
                       const float* const* tables, int32_t n_types, int32_t K, int64_t n_rows,
                       float* S, float* wsum, int64_t ld_s, int64_t ld_w, hipStream_t stream);

/* The mean aggregation of a sampled block in the strided layout (regnn_ns_hop strided = 1: row
 * i's edges at slots [i S, i S + cnt[i]], the self loop last; ABI 44): y[i] = inv[i] sum_e
 * tab[rel_e] x[idx_e] + bias for i < live[0], bias (or 0) past it, over n_rows (the capacity)
 * rows of F fp32 features (F % 4 == 0, F <= 1024; x, y, bias 16-byte aligned); rel_table may be
 * NULL (weight 1). What regnn_spmm_fwd computes over the same block in the CSR layout, summed
 * in the same slot order (mag/regnn_layers.py:110-148). */
int regnn_ns_spmm_strided_fwd(const int32_t* live, const int32_t* cnt, int32_t stride,
                              const int32_t* idx, const uint8_t* rel, const float* rel_table,
                              const float* inv, const float* bias, const float* x, float* y,
                              int64_t n_rows, int32_t F, hipStream_t stream);

/* Layer 0's [S | w | 0] operand from the sampler's per-type input sums (relation slots; ABI 44):
 * the outputs of regnn_ns_hop_typed_sums for hop `hop` (U [cap][T][K] unweighted sums, cnt
 * [cap][T] counts, x_self [cap][K], u_rel [cap][T + 1]: each slot's relation or -1, then the self
 * loop's relation n_et + node type) and the relation table tab give, for rows v < sizes[hop],
 *   out[v][t K ..] = tab[u_rel[v][t]] U[v][t] + [t = u_rel[v][T] - n_et] tab[u_rel[v][T]] x_self[v]
 *   out[v][T K + t] = tab[u_rel[v][t]] cnt[v][t] + [same] tab[u_rel[v][T]]     (0 past T, < Tp)
 * what regnn_ns_typed_agg forms from the sampled edges (mag/regnn_layers.py:110-129), with Tp = T
 * rounded up to 4; rows [sizes[hop], next multiple of 128) are zeros, later rows untouched.
 * K = 128, T <= 4, ld >= T K + Tp. The backward writes slab[b][r] (slab_rows blocks; reduce with
 * regnn_rel_reduce) of d tab[r] = sum over r's slots of <U, gS> + cnt gw and over r's self loops
 * of <x_self, gS_t_self> + gw_t_self: fixed order, bitwise reproducible. */
int regnn_ns_slot_agg(const int32_t* sizes, int32_t hop, const float* U, const float* cnt,
                      const float* x_self, const int32_t* u_rel, const float* rel_table,
                      int32_t n_et, int32_t n_types, int32_t K, int64_t cap, float* out,
                      int64_t ld, hipStream_t stream);
int regnn_ns_slot_agg_bwd(const int32_t* sizes, int32_t hop, const float* U, const float* cnt,
                          const float* x_self, const int32_t* u_rel, const float* g, int64_t ld,
                          int32_t n_et, int32_t n_types, int32_t K, float* slab, int32_t n_rel,
                          int32_t slab_rows, hipStream_t stream);

/* Relation-table gradient of regnn_ns_typed_agg: slab[b][r] = block b's partial of
 * sum_{e: rel_e = r} (<tables[t_e][row_e], gS[v][t_e]> + gw[v][t_e]) (per row group bins added
 * in entry order, the groups in a fixed order: bitwise reproducible). Launches slab_rows blocks;
 * reduce the slab with regnn_rel_reduce. n_rel <= 256. */
int regnn_ns_typed_agg_bwd(const int32_t* ptr, const int32_t* idx, const uint8_t* rel,
                           const int32_t* n_id, const int32_t* ntype, const int64_t* local,
                           const int32_t* e_type, const int64_t* e_off,
                           const float* const* tables, int32_t n_types, int32_t K, int64_t n_rows,
                           const float* gS, const float* gw, int64_t ld_s, int64_t ld_w,
                           float* slab, int32_t n_rel, int32_t slab_rows, hipStream_t stream);


/* ---------------------------------------------------------------------------------------
 * Fused NS model step: the REGNN of mag/regnn_ns.py:216-346 (model 'regcn', self_loop_type 2,
 * use_norm 'ln', residual off, feats_type != 2, hidden 64) forward + nll_loss + backward over the
 * blocks regnn_ns_hop wrote, with no host sizes (every kernel reads the counts in `sizes`).
 * Replaces, per step (mag/regnn_ns.py:399-406): group_input's per-type Linear (:300-326), each
 * REGCNConv (x @ W, relation-table mean aggregation + bias, LayerNorm; mag/regnn_layers.py:
 * 80-150), relu + dropout (:341-343), out_lin + log_softmax (:345-346), F.nll_loss (:404) and
 * loss.backward() (:405), writing every parameter gradient into caller-provided buffers.
 *
 * Arithmetic (fp32 throughout): the group_input Linear and the first conv's weight are applied
 * as one composed map x @ (W_t^T W_0) + b_t W_0 (associativity; the gradients of W_t, b_t and W_0
 * follow by the chain rule), after layer 0's aggregation (linearity: the input rows are summed
 * per target row and source type, then projected). Dropout masks are this build's hash
 * (regnn_spmm_fwd_dropout's spec) keyed on s = mix64(state[0] ^ mix64((state[1] << 40) ^
 * (state[3] << 8) ^ (layer + 0x51ED27))) (seed, epoch, global batch), row = target row of the
 * layer's block, 4 features per 16-byte vector.
 *
 * L = 2 (the reference's default num_layers; C <= 384): 5 launches (6 without rel_slots), the
 * group_input Linear and each conv's x @ W applied after their layer's aggregation (linearity:
 * mean_e(ew x_e) W = mean_e(ew x_e W)), the transposed aggregation of layer 1 as 2^-40
 * fixed-point integer sums, every other reduction fixed-order: the step is bitwise
 * reproducible; optionally the Adam update of regnn_nsm_work.adam in the last launch.
 * L = 3, 4 (or C > 384): the composed-map form above, 8+ launches, layer >= 1 transposed
 * aggregations with float atomics (as regnn_ns_spmm_bwd).
 * --------------------------------------------------------------------------------------- */
#define REGNN_NSM_MAX_TYPES 8
#define REGNN_NSM_MAX_LAYERS 4

typedef struct regnn_nsm_params {
    int32_t n_types;          /* node types T (x_dict keys 0..T-1), <= 8 */
    int32_t k_in;             /* input feature width: 64 or 128, T * (k_in + 1) <= 600 */
    int32_t n_layers;         /* L in [2, 4]; layer l reads hop L-1-l's block */
    int32_t n_classes;        /* C <= 448 */
    float alpha;              /* scaling_factor (mag/regnn_layers.py:110) */
    float p_drop;             /* dropout after each conv's relu (training), in [0, 1) */
    int32_t n_rel[REGNN_NSM_MAX_LAYERS];  /* len(relation_weight) per layer, <= 64 */
    const float* x_tab[REGNN_NSM_MAX_TYPES];  /* x_dict[t] [n_t, k_in], rows = local_node_idx */
    const float* lin_w[REGNN_NSM_MAX_TYPES];  /* lins[t].weight [64, k_in] */
    const float* lin_b[REGNN_NSM_MAX_TYPES];  /* lins[t].bias [64] */
    const float* conv_w[REGNN_NSM_MAX_LAYERS];  /* convs[l].weight [64, 64] (x @ W) */
    const float* conv_b[REGNN_NSM_MAX_LAYERS];
    const float* conv_rw[REGNN_NSM_MAX_LAYERS]; /* convs[l].relation_weight [n_rel] */
    const float* ln_w[REGNN_NSM_MAX_LAYERS];
    const float* ln_b[REGNN_NSM_MAX_LAYERS];
    const float* out_w;       /* out_lin.weight [C, 64] */
    const float* out_b;       /* out_lin.bias [C] */
    float* g_lin_w[REGNN_NSM_MAX_TYPES];
    float* g_lin_b[REGNN_NSM_MAX_TYPES];
    float* g_conv_w[REGNN_NSM_MAX_LAYERS];
    float* g_conv_b[REGNN_NSM_MAX_LAYERS];
    float* g_conv_rw[REGNN_NSM_MAX_LAYERS];
    float* g_ln_w[REGNN_NSM_MAX_LAYERS];
    float* g_ln_b[REGNN_NSM_MAX_LAYERS];
    float* g_out_w;
    float* g_out_b;
    float* loss;              /* [1]: mean nll over the batch targets with a label >= 0 */
    int32_t n_edge_types;     /* relations < n_edge_types are edges; n_edge_types + type: self loops */
    int32_t rel_slots;        /* 1: every (target type, source type) pair has at most one edge
                                 relation (the caller checked the graph once): layer 0 sums its
                                 rows per source type unweighted and the relation-table gradient
                                 comes from those sums (no second pass over the edges; needs
                                 u_self / u_rel); 0: the edge pass */
    int32_t two_layer;        /* 1: the caller set up the two-layer form (L = 2, C <= 384, hop 0's
                                 edge capacity <= 32768, regnn_nsm_work.p0 / gh1 / csc_* set):
                                 regnn_nsm_step and regnn_nsm_slab_floats take that form only
                                 then, one decision for both; 0: the composed-map form (ABI 36) */
} regnn_nsm_params;

typedef struct regnn_nsm_work {
    const int64_t* state;     /* regnn_ns_batch / regnn_ns_hop state (reads [0] and [4]) */
    const int32_t* sizes;     /* regnn_ns_hop sizes */
    const int32_t* n_id;      /* [cap[L]] int32 */
    int32_t cap[REGNN_NSM_MAX_LAYERS + 1];    /* capacity of n_id after h hops */
    const int32_t* blk_ptr[REGNN_NSM_MAX_LAYERS];   /* hop h's block (regnn_ns_hop output) */
    const int32_t* blk_idx[REGNN_NSM_MAX_LAYERS];
    const uint8_t* blk_rel[REGNN_NSM_MAX_LAYERS];
    const float* blk_inv[REGNN_NSM_MAX_LAYERS];
    const int32_t* ntype;     /* node type per global node */
    const int64_t* local;     /* local_node_idx per global node */
    const int64_t* labels;    /* label per global node (< 0: none) */
    /* scratch, caller-allocated (sizes in rows of 64 floats unless noted) */
    float* wc;                /* T * (k_in + 1) * 64 floats: the composed first map */
    float* gwc;               /* same size: its gradient */
    float* tabs;              /* L * 64 floats */
    float* xs[REGNN_NSM_MAX_LAYERS];    /* layer l >= 1's source rows: cap[L-l] rows ([0] unused) */
    float* gxs[REGNN_NSM_MAX_LAYERS];   /* their gradient: cap[L-l] rows ([0] unused) */
    float* a[REGNN_NSM_MAX_LAYERS];     /* layer l < L-1: pre-LayerNorm rows, cap[L-1-l] rows */
    float* stats[REGNN_NSM_MAX_LAYERS]; /* layer l < L-1: (mean, rstd), 2 * cap[L-1-l] floats */
    float* ga[REGNN_NSM_MAX_LAYERS];    /* d loss / d pre-LN rows: cap[L-1-l] rows */
    /* layer 0 (target rows of hop L-1's block, cap[L-1] of them; E1 = that block's edge capacity) */
    const int32_t* edge_type; /* E1: regnn_ns_hop's edge_type output for hop L-1 */
    const int64_t* edge_off;  /* E1: its edge_off output */
    float* s_agg;             /* cap[L-1] * T * k_in: per-type weighted input sums of each row */
    float* s_w;               /* cap[L-1] * T: per-type sums of the relation weights */
    float* z;                 /* cap[L-1] * T * k_in: W_c[t] (inv ga) per row and type */
    float* beta;              /* cap[L-1] * T */
    float* nvalid;            /* 1 float: labelled targets of the batch */
    float* slab;              /* regnn_nsm_slab_floats() floats of per-block partials */
    float* u_self;            /* rel_slots: cap[L-1] * k_in, each row's self-loop input row */
    int32_t* u_rel;           /* rel_slots: cap[L-1] * (T + 1), relation of each source-type slot */
    /* the two-layer step (L = 2, C <= 384, hop 0's edge capacity <= 32768): */
    float* p0;                /* cap[1] * 64: layer 0's group_input projection, summed per row */
    const struct regnn_nsm_adam* adam;   /* NULL, or the optimizer the last launch applies */
    float* gh1;               /* cap[0] * 64: G W_1^T of layer 1's target rows (its transposed pass) */
    const int32_t* csc_ptr0;  /* hop 0's transposed index (regnn_ns_hop csc_ptr / csc_ent / */
    const int32_t* csc_ent0;  /* csc_long) */
    const int32_t* csc_long0;
    int32_t stride[REGNN_NSM_MAX_LAYERS];        /* per hop: 0 = CSR block, else its fixed stride */
    const int32_t* blk_cnt[REGNN_NSM_MAX_LAYERS]; /* per hop (strided): sampled edges per row */
    int32_t part;             /* two-layer step: 0 = every launch; 1 = the forward, the head and
                                 layer 1's transposed pass (agg0, head, gather); 2 = the rest
                                 (bwd0, rel0, finalize). A caller orders other work between the
                                 two parts (NSTrainer joins the sampler stream there). */
    /* two-layer step: layer 1's transposed pass gives each piece of a hub row (> 16 entries,
     * the csc_long0 piece table) a workgroup of its own; the pieces' exact 2^-40 fixed-point
     * sums meet in hub_acc, the last piece of a row (hub_ticket) finishes it. hub_ticket and
     * hub_terms zero-filled once by the caller, left zero by every step; hub_terms[192] is the
     * step's fixed-point overflow flag (a term past 2^8: that step's loss reads NaN). */
    unsigned long long* hub_acc;   /* REGNN_CSC_LONG_MAXPIECE * 64 */
    int32_t* hub_ticket;           /* REGNN_CSC_LONG_CAP */
    unsigned long long* hub_terms; /* 3 * 64 + 1 */
    int32_t split_finalize;   /* two-layer step, adam NULL: 1 = part 1 ends with the reduction of
                                 the gradients final after layer 1's transposed pass (out_lin,
                                 layer 1, layer 0's conv bias and LayerNorm), part 2 reduces the
                                 rest (a caller all-reduces the first set while part 2 runs) */
    int32_t pre_sums;         /* two-layer step with rel_slots, k_in 128, T <= 4: 1 = s_agg / s_w /
                                 u_self / u_rel already hold the batch's layer-0 input sums
                                 (regnn_ns_hop_typed_sums): layer 0 reads them instead of
                                 gathering its input rows (ABI 41) */
} regnn_nsm_work;

/* Adam over the flat parameter bucket whose gradient bucket starts at grad_base (every g_*
 * pointer of regnn_nsm_params a view into it; gradients outside [grad_base, grad_base + n) are
 * written but not stepped): regnn_adam_flat's arithmetic and step counter, applied by the
 * two-layer step's last launch right after each gradient element's reduction (one rank: no
 * all-reduce between the backward and the update). */
typedef struct regnn_nsm_adam {
    float* param;
    float* exp_avg;
    float* exp_avg_sq;
    const float* grad_base;
    int64_t n;
    float lr, beta1, beta2, eps, weight_decay, grad_scale;
    int64_t* step;      /* advanced once per step by the launch before the update (device) */
    uint32_t* ticket;   /* unused by regnn_nsm_step since ABI 35 (kept: the struct's layout) */
} regnn_nsm_adam;

/* Floats of the per-block partial slab regnn_nsm_step needs for these parameters and a batch
 * capacity cap0 (= regnn_nsm_work.cap[0]). */
int64_t regnn_nsm_slab_floats(const regnn_nsm_params* p, int32_t cap0);

/* One forward + loss + backward of the model over the current batch (after regnn_ns_batch and
 * the L regnn_ns_hop calls of the step): writes every g_* buffer (overwritten, not accumulated)
 * and *loss (and, with w->adam, updates the parameters). 5 kernel launches for L = 2 with
 * rel_slots (L in [2, 4]), none of them sized from the host. */
int regnn_nsm_step(const regnn_nsm_params* p, const regnn_nsm_work* w, hipStream_t stream);

/* Adam step over flat buffers (replaces torch.optim.Adam.step, mag/regnn_ns.py:407, for
 * parameters laid out in one flat bucket): with weight decay wd the gradient is g + wd * p
 * (torch's L2 form; g = grad_scale * grad, e.g. 1 / ranks after a SUM all-reduce, so the
 * data-parallel mean needs no separate pass), t = *step + 1, m = lerp(m, g, 1 - beta1), v = beta2 v + (1 - beta2) g^2,
 * p -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps). *step (int64) and *ticket
 * (uint32, zero-filled once) live on the device; the launch advances *step itself, so a
 * captured graph needs no host update. ticket NULL (ABI 44): *step was already advanced by the
 * caller (t = *step, nothing written): no end-of-launch ticket, whose one contended atomic per
 * workgroup serialises the tail of a large bucket's launch. */
int regnn_adam_flat(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                    float lr, float beta1, float beta2, float eps, float weight_decay,
                    float grad_scale, int64_t* step, uint32_t* ticket, hipStream_t stream);

/* ---- fp32-accurate dense GEMM on bf16 MFMA (bf16x6) ----------------------------------------
 * C = op(A) op(B) (+ beta C), M x N x K, row-major fp32: trans_a: A stored [K][M] (lda >= M),
 * else [M][K] (lda >= K); trans_b: B stored [N][K], else [K][N]. Each operand is split into three
 * bf16 parts and the six significant cross products accumulate in fp32 (error ~ fp32 rounding).
 * Replaces the wide NS model's torch.mm / addmm / nn.Linear products (mag/regnn_ns.py:300-346,
 * mag/regnn_layers.py:101-107 at hidden 128 .. 512) and their backward products. Operands whose
 * contiguous dimensions (K or M for A, K or N for B) and lda / ldb are multiples of 4 and whose
 * bases are 16-byte aligned load 16-byte vectors, any others per element. splits > 1: split-K over `work` (regnn_gemm_x6_work_floats floats), partials
 * added in split order (bitwise reproducible). */
int64_t regnn_gemm_x6_work_floats(int64_t M, int64_t N, int32_t splits);
int regnn_gemm_x6(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                  const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                  float beta, float* work, int32_t splits, const int32_t* m_live,
                  const int32_t* k_live, hipStream_t stream);
/* m_live / k_live (ABI 41; device int32 counts, may be NULL): op(A)'s rows m >= *m_live, and the
 * k >= *k_live columns of op(A) / rows of op(B), are zero (the unused rows of a capacity-sized
 * sampled block): the kernel skips their products (C rows >= *m_live get beta C) -- the same C,
 * with the work of the live rows only. With m_live and splits == 1 the launch uses 64-row tiles
 * (twice the live tiles; env REGNN_GEMM_BM64=off: 128): every C element sums the same k-steps and
 * products in the same order, so the bits are those of the 128-row tiling. */

/* Several strided 2-D fp32 copies in one launch: dst[i * cols + j] = src[i * s0 + j * s1] for
 * each descriptor (the module path's parameter gradients, some of them transposed views, into the
 * flat gradient bucket: one launch instead of one copy per parameter). */
typedef struct regnn_copy2d {
    const float* src;
    float* dst;
    int64_t rows, cols, s0, s1;
} regnn_copy2d;
int regnn_copy2d_many(const regnn_copy2d* d, int32_t n, hipStream_t stream);

/* ---- The wide NS model's per-layer epilogue (mag/regnn_layers.py:131-135 + mag/regnn_ns.py:
 * 341-343 at hidden H in {64, 128, 256, 512, 1024}) ----------------------------------------------
 * Forward over n rows of H fp32: a = rs[v] x[v] + bias (+ res[v]) (rs, bias, res optional), y =
 * dropout(relu(LayerNorm(a; gamma, beta, eps 1e-5))); writes a, stats [n][2] = (mean, rstd) and
 * y. Dropout (p_drop > 0): the fused NS step's mask spec (regnn_nsm_step) keyed on the sampler
 * state and `layer`. Backward from gy: gx = rs[v] d a (rs NULL: 1), gres = d a (optional), and
 * slab [regnn_wide_ln_slab_rows(n, H)][3 H] of per-block partials [sum d a | sum gy' xhat | sum
 * gy'] (the bias, LN weight and LN bias gradients after regnn_rel_reduce). 16-byte aligned rows.
 * live (ABI 46; device int32 count, may be NULL): only rows v < *live are read (a capacity-sized
 * sampled block whose later rows nothing reads): the forward leaves a / stats / y past it as they
 * were, the backward writes zeros to gx (and gres) there and skips those rows' partials (exact
 * zeros for zero gy). */
int regnn_wide_ln_fwd(int64_t n, int32_t H, const float* x, const float* rs, const float* bias,
                      const float* res, const float* gamma, const float* beta,
                      const int64_t* state, int32_t layer, float p_drop, float* a, float* stats,
                      float* y, const int32_t* live, hipStream_t stream);
int64_t regnn_wide_ln_slab_rows(int64_t n, int32_t H);
int regnn_wide_ln_bwd(int64_t n, int32_t H, const float* gy, const float* a, const float* stats,
                      const float* rs, const float* gamma, const float* beta,
                      const int64_t* state, int32_t layer, float p_drop, float* gx, float* gres,
                      float* slab, const int32_t* live, hipStream_t stream);

/* ---- Per-node-type input rows of the ogbn-mag path (mag/regnn_ns.py:300-326, group_input) ----
 * The reference builds the batch's input matrix with one boolean mask per node type (a host
 * sync each) and, for feats_type != 2, runs each type's Linear over its masked subset. Node i of
 * the batch is n_id[i] (n_id NULL: i), of type node_type[n_id[i]] with row local_idx[n_id[i]]
 * in its type's table (both int64, per global node). Tables are fp32 [*, K] row-major,
 * 16-byte aligned, indexed by node type (T <= 8).
 *
 * regnn_typed_gather: out[i] = tab[type][local] (NULL table or type outside [0, T): zeros, as
 * regnn_ns.py:307's zero matrix), out [n, K] fp32 (feats_type 2: the shared self.lin follows).
 * regnn_typed_scatter: gtab[type][local] += g[i] for the tables that learn (NULL: skipped) —
 * the backward of the gather into feats_type-2 embedding tables (float atomics; rows of one
 * batch are distinct, so each element receives one add). */
int regnn_typed_gather(const int64_t* n_id, int64_t n, const int64_t* node_type,
                       const int64_t* local_idx, int32_t T, const float* const* tab, int32_t K,
                       float* out, hipStream_t stream);
int regnn_typed_scatter(const int64_t* n_id, int64_t n, const int64_t* node_type,
                        const int64_t* local_idx, int32_t T, float* const* gtab, int32_t K,
                        const float* g, hipStream_t stream);

/* Per-type Linear fused with the gather (feats_type != 2: lins[t] per node type). The n rows
 * come sorted by type (a stable sort, built on the device by the caller): entry i is output row
 * order[i], reading row src[i] of its type's table; type t's run is [type_off[t], type_off[t+1])
 * (type_off int32 [T+1] on the device: the launch reads the run sizes itself, no host sync).
 *   fwd:   Y[order[i]] = tab[t][src[i]] W[t]^T + b[t]        W[t] [O, K], b[t] [O] or NULL
 *   wgrad: gW[g] = sum over types t with wgroup[t] = g of sum_i gY[order[i]]^T tab[t][src[i]],
 *          gb[g] (NULL: skipped) the matching sums of gY rows; per-chunk partials in `slab`
 *          (regnn_typed_slab_floats(n, T, K, O) floats, no zeroing needed) reduced in fixed
 *          chunk order (deterministic).
 * Host arrays tab / W / b hold T device pointers, gW / gb G, wgroup T ints. fp32 MFMA
 * (v_mfma_f32_16x16x4_f32: exact fp32 products). K in {64, 128, 256}; O a multiple of 16
 * (fwd) / 64 (wgrad), else REGNN_EUNSUPPORTED. */
int64_t regnn_typed_chunks(int64_t n, int32_t T, int32_t rows);
int64_t regnn_typed_slab_floats(int64_t n, int32_t T, int32_t K, int32_t O);
int regnn_typed_linear_fwd(const int64_t* order, const int64_t* src, const int32_t* type_off,
                           int64_t n, int32_t T, const float* const* tab, const float* const* W,
                           const float* const* b, int32_t K, int32_t O, float* Y,
                           hipStream_t stream);
int regnn_typed_linear_wgrad(const int64_t* order, const int64_t* src, const int32_t* type_off,
                             int64_t n, int32_t T, const float* const* tab, const int32_t* wgroup,
                             int32_t G, int32_t K, int32_t O, const float* gY, float* slab,
                             float* const* gW, float* const* gb, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* REGNN_HIP_H */
