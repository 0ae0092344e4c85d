/*
 * dw_hip.h — C ABI of the MI355X (gfx950) DeepWalk / node2vec hot path.
 *
 * The reference (Robotmurlock/Deepwalk-and-Node2vec) is pure Python and has no FFI; each entry
 * point below replaces one Python call surface of its two hot paths:
 *
 *   path A (walks):  shallow_encoders/graph/random_walk_generator.py:41-119
 *   path B (SGNS):   shallow_encoders/word2vec/model.py:79-91, loss.py:14-22,
 *                    utils/sampling.py:7-21, trainer.py:131-152, + torch.optim.Adam step
 *
 * Conventions (every function):
 *   - all array arguments are DEVICE pointers owned by the caller (torch tensors' data_ptr());
 *     no function allocates user-visible memory;
 *   - `stream` is a hipStream_t passed as void* (torch.cuda.current_stream().cuda_stream);
 *     every launch is stream-ordered and asynchronous;
 *   - functions are stateless and reentrant (distinct buffers ⇒ safe from several host threads);
 *   - return value: DW_OK (0) or a negative DW_E_* code; dw_last_error_string() (thread-local)
 *     describes the last failure. Nothing throws or aborts across the ABI;
 *   - conditions found ON THE DEVICE (an isolated node met by a walker, a rejection loop that
 *     exceeded its bound, a bad CSR entry) are OR-ed into the caller's int32 `status` word
 *     (DW_S_* bits) so the host can check them when it next synchronises.
 *
 * Graph layout in HBM (CSR, vocabulary ids: row 0 is `<unk>` with no neighbours, node i of the
 * vocabulary is row i; neighbour order = networkx `graph.neighbors()` insertion order):
 *   row_ptr int64[n_rows+1], col int32[nnz], weights float64[nnz] (NULL = unweighted),
 *   col_sorted int32[nnz] (each row's neighbours sorted ascending, for adjacency tests).
 */
#ifndef DW_HIP_H
#define DW_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---------------------------------------------------------------------- */
#define DW_OK                0
#define DW_E_INVALID_ARG    -1
#define DW_E_HIP            -2
#define DW_E_UNSUPPORTED    -3

/* ---- device status bits (OR-ed into the caller's int32 status word) -------------------- */
#define DW_S_ISOLATED_NODE   1   /* walker reached a node with no neighbours (reference: IndexError) */
#define DW_S_ZERO_WEIGHT     2   /* all neighbour weights zero (reference: ZeroDivisionError)        */
#define DW_S_REJECTION_CAP   4   /* node2vec rejection exceeded DW_MAX_REJECTION_ROUNDS              */
#define DW_S_BAD_CSR         8   /* row_ptr not monotone / col out of range                          */
#define DW_S_BAD_INDEX      16   /* an index outside [0, V) reached the SGNS kernel                  */
#define DW_S_RECORDS_FULL   32   /* owner-form SGNS records exceeded the workspace (not expected)    */
#define DW_S_DUP_NEIGHBOR   64   /* a CSR row lists a neighbour twice (dw_csr_check_simple)          */
#define DW_S_FIXED_RANGE   128   /* a gradient term past the deterministic fixed-point range         */

#define DW_METHOD_DEEPWALK   0   /* random_walk_generator.py:56-72 ('deepwalk' and 'dfs')          */
#define DW_METHOD_NODE2VEC   1   /* random_walk_generator.py:75-119                                  */

#define DW_MAX_REJECTION_ROUNDS 65536
#define DW_ADJ_HASH_MIN_DEG  8   /* rows of higher degree get an adjacency hash (dw_adj_hash_*)        */

/* ---- library ---------------------------------------------------------------------------- */
const char *dw_last_error_string(void);
int dw_abi_version(void);               /* bumps on any signature change */
/* SHA-256 prefix (16 hex digits) of the sources the library was built from (csrc/build.py
 * source_id): a shipped binary can be checked against the tree it came with. */
const char *dw_build_id(void);
int dw_device_sync(void *stream);       /* hipStreamSynchronize(stream); used by the host mirror */
/* dst = src, bytes a multiple of 16 (16-B aligned device buffers): a STREAM-copy kernel, the
 * measured HBM roofline bench.py reports beside the spec peak. */
int dw_stream_copy(const void *src, void *dst, int64_t bytes, void *stream);

/* Host-side (no device work): CPython 3.10 random.shuffle over range(n), bit for bit — the
 * reference's start-node shuffle (datasets.py:45,86-88) in native code. mt_state: the 625 words
 * of random.getstate()[1] (624-word MT19937 state + index), advanced in place exactly as
 * Python's shuffle would; perm: int64[n] out. */
int dw_host_shuffle(uint32_t *mt_state, int64_t *perm, int64_t n);

/* ---- the reference's uniform stream on the device ------------------------------------------
 * CPython's random.random() (Modules/_randommodule.c: MT19937 + genrand_res53), the one draw per
 * walk step of random_walk_generator.py:68,113 (random.choices(..., k=1)); replaces the host
 * draw + H2D copy in front of dw_walk_replay(_inline). Replaces, in the reference,
 * `random.random()` called n times on the global generator (datasets.py:87-91 -> walk()).
 *
 * dw_mt_jump_table (HOST, no device work): jump-ahead polynomials for dw_mt_uniforms. Chain c
 * (c >= 1) of a call starts at raw word 624*window_stride*c of the generator's sequence; its
 * entry lists the exponents l (ascending) of t^(624*window_stride*c - 2) mod phi(t), phi =
 * MT19937's characteristic polynomial (degree 19937, 135 terms). offsets: int64[n_chains+1]
 * (chain c's exponents are positions[offsets[c] .. offsets[c+1])); positions: uint16[capacity]
 * (n_chains * 19937 always suffices; DW_E_INVALID_ARG when too small). Host buffers.
 *
 * dw_mt_uniforms: out[k] = the (k+1)-th random.random() of the generator whose state is
 * (mt[0..623], index) — random.getstate()[1] — for k < n; state_out (625 words: array + index)
 * receives the state after the n draws, for random.setstate. mt, out, state_out, jump_pos,
 * jump_off, workspace: DEVICE buffers (jump_*: a dw_mt_jump_table of the same window_stride
 * with at least chains = ceil(windows / window_stride) entries, windows = (index + 2n - 1) / 624
 * + 1; workspace: dw_mt_workspace_words(chains) uint32 words; all may be NULL when that is one
 * chain). Two stream-ordered launches: the chains' jumps, then one workgroup per chain. */
int dw_mt_jump_table(int64_t window_stride, int64_t n_chains, int64_t *offsets,
                     uint16_t *positions, int64_t capacity);
int dw_mt_uniforms(const uint32_t *mt, int32_t index, int64_t n, double *out,
                   uint32_t *state_out, int64_t window_stride, const uint16_t *jump_pos,
                   const int64_t *jump_off, int64_t n_chains_table, uint32_t *workspace,
                   int64_t workspace_words, void *stream);
int64_t dw_mt_workspace_words(int64_t n_chains);

/* A generator whose state lives in HBM (state: 625 uint32 words, the 624-word array + the
 * index, random.getstate()[1]'s layout; torch's CPU generator maps onto the same layout), advanced
 * in place by n draws (through scratch, 625 words, then copied back; stream-ordered and
 * capturable in a HIP graph):
 *   mode 0: out float64[n] = the next n random.random() (as dw_mt_uniforms);
 *   mode 1: out int64[n] = the next n torch.randint(0, range, ...) values of torch's CPU
 *           generator for range < 2^28 (aten's mt19937, one 32-bit output per value,
 *           `% range`) — generate_noise_batch (utils/sampling.py:7-21), noise='torch';
 *   mode 2: the same for 2^28 <= range < 2^32, where torch takes two outputs per value
 *           ((first << 32 | second) % range).
 * index >= 0: the host knows the index (it must equal state[624]), the launch is sized to it;
 * index < 0: read on the device (a replayed graph), the launch covers the largest index.
 * jump_* / workspace as dw_mt_uniforms for chains = ceil(windows / window_stride), windows =
 * (index + w n - 1) / 624 + 1, w = 1 (mode 1) or 2, index = 624 when read on device. */
int dw_mt_draw(int32_t mode, uint32_t *state, int32_t index, int64_t n, void *out,
               uint64_t range, uint32_t *scratch, int64_t window_stride,
               const uint16_t *jump_pos, const int64_t *jump_off, int64_t n_chains_table,
               uint32_t *workspace, int64_t workspace_words, void *stream);

/* ---- graph ------------------------------------------------------------------------------- */

/* Validate a CSR on the device: row_ptr[0]==0, monotone, row_ptr[n_rows]==nnz, 0<=col<n_rows.
 * Replaces nothing in the reference (networkx guarantees it); guards every kernel below. */
int dw_csr_validate(const int64_t *row_ptr, const int32_t *col, int64_t n_rows, int64_t nnz,
                    int32_t *status, void *stream);

/* Sorted copy of every neighbour list (ascending ids), used for the node2vec adjacency test
 * `prev_node in candidate_neighbors` (random_walk_generator.py:106-107).
 * Two-phase temp-storage protocol: call with temp==NULL to get *temp_bytes, then again. */
int dw_csr_sort_copy(const int64_t *row_ptr, const int32_t *col, int64_t n_rows, int64_t nnz,
                     int32_t *col_sorted, void *temp, size_t *temp_bytes, void *stream);

/* Sets DW_S_DUP_NEIGHBOR in status when a row of col_sorted (dw_csr_sort_copy) holds two equal
 * entries. The reference's networkx.Graph keeps one entry per neighbour
 * (random_walk_generator.py:41-42 lists graph.neighbors(node)), and the bit-exact node2vec replay
 * relies on it (one position of prev in N(v), class counts by intersection), so the host refuses a
 * non-simple CSR there. */
int dw_csr_check_simple(const int64_t *row_ptr, const int32_t *col_sorted, int64_t n_rows,
                        int64_t nnz, int32_t *status, void *stream);

/* Per-row adjacency hash for the fast node2vec walker's test `prev_node in
 * candidate_neighbors` (random_walk_generator.py:106-107): one probe of a 64-B bucket instead of
 * a ceil(log8 deg)-load search of the sorted list. A row u of degree > DW_ADJ_HASH_MIN_DEG owns
 * nb = ceil(4 deg / 48) buckets of 16 int32 slots (load <= 3/4) at adj_hash + adj_off[u]; rows
 * of lower degree own none (their neighbour list itself is one load).
 *   dw_adj_hash_offsets: adj_off int64[n_rows + 1] (exclusive scan of the per-row slot counts;
 *     adj_off[n_rows] = total slots). Two-phase temp protocol as dw_csr_sort_copy.
 *   dw_adj_hash_build: fills adj_hash int32[n_slots] (n_slots = adj_off[n_rows]). */
int dw_adj_hash_offsets(const int64_t *row_ptr, int64_t n_rows, int64_t *adj_off, void *temp,
                        size_t *temp_bytes, void *stream);
int dw_adj_hash_build(const int64_t *row_ptr, const int32_t *col, int64_t n_rows,
                      const int64_t *adj_off, int64_t n_slots, int32_t *adj_hash, int32_t *status,
                      void *stream);
/* adj_hpos int32[n_slots]: for every filled slot of adj_hash, the index of its key in the row's
 * neighbour order (-1 for free slots) — the bit-exact node2vec replay's position lookups
 * (dw_walk_replay_indexed). After dw_adj_hash_build. */
int dw_adj_hash_positions(const int64_t *row_ptr, const int32_t *col, int64_t n_rows,
                          const int64_t *adj_off, const int32_t *adj_hash, int64_t n_slots,
                          int32_t *adj_hpos, int32_t *status, void *stream);

/* Per-row Vose alias tables for first-order weighted sampling (the fast-mode replacement of
 * get_node_normalized_edge_weights + random.choices, random_walk_generator.py:50-53,68).
 * prob_thr[e] = floor(P_accept * 2^32) clamped to [0, 2^32-1] with 2^32-1 meaning "always";
 * alias[e] = local index (0..deg-1) of the alias entry.
 * work_prob float64[nnz], work_idx int32[nnz]: caller-provided scratch. */
int dw_alias_build(const int64_t *row_ptr, const double *weights, int64_t n_rows, int64_t nnz,
                   uint32_t *prob_thr, int32_t *alias, double *work_prob, int32_t *work_idx,
                   int32_t *status, void *stream);

/* ---- walks -------------------------------------------------------------------------------- */

/* ---- Graph ingestion on the device (shallow_encoders/graph/rmat.py) ----
 * R-MAT edge draws replacing rmat.py:rmat_edges' numpy loop: the uniforms are numpy's
 * default_rng PCG64 stream, draw index level * n_edges + edge. The host supplies level_state
 * (2*scale uint64: lo, hi of the 128-bit state before level l's first draw), jump (64 x 4
 * uint64: multiplier lo/hi, increment lo/hi of 2^i steps), the stream increment and the
 * thresholds t1 = a, t2 = a + b, t3 = a + b + c. Output: edges packed (src << 32 | dst),
 * self-loops dropped, undirected duplicates removed keeping the first draw, in draw order;
 * *n_unique (device int64) = their count. Workspace >= dw_ingest_workspace_bytes. */
int dw_ingest_workspace_bytes(int32_t scale, int64_t n_edges, int64_t n_nodes, size_t *bytes);
int dw_rmat_edges(int32_t scale, int64_t n_edges, const uint64_t *level_state,
                  const uint64_t *jump, uint64_t inc_lo, uint64_t inc_hi, double t1, double t2,
                  double t3, uint64_t *edges, int64_t *n_unique, void *workspace,
                  size_t workspace_bytes, void *stream);

/* Nodes of [0, n_nodes) that no edge touches, increasing (rmat.py's isolated-node patch list);
 * *n_isolated is a device int64. Endpoints >= n_nodes set DW_S_BAD_CSR. */
int dw_graph_isolated(const uint64_t *edges, int64_t n_edges, int64_t n_nodes,
                      int32_t *isolated, int64_t *n_isolated, int32_t *status, void *workspace,
                      size_t workspace_bytes, void *stream);

/* CSR of an undirected packed edge list (rmat.py:csr_from_edges / networkx add_edges_from
 * order): row_ptr int64 [n_nodes + 2] (row 0 = <unk>, row i+1 = node i), col int32
 * [2 n_edges] holding vocabulary ids (node + 1); each row lists its edges in edge order. */
int dw_csr_from_edges(const uint64_t *edges, int64_t n_edges, int64_t n_nodes,
                      int64_t *row_ptr, int32_t *col, int32_t *status, void *workspace,
                      size_t workspace_bytes, void *stream);

/* Exact replay walker — bit-exact with DeepWalk.walk / Node2Vec.walk
 * (random_walk_generator.py:61-72 / 94-119) given the uniforms random.random() would return.
 * uniforms: float64[n_walks, L-1], consumed in the reference's order (one per step).
 * out: int32[n_walks, L]. Weighted graphs: weights != NULL (float64, networkx 'weight').
 * Arithmetic follows CPython 3.10 exactly: left-to-right fp64 sum, w *= (1/p), w/sum,
 * itertools.accumulate, total = cum[-1] + 0.0, bisect_right(cum, u*total, 0, deg-1).
 * Unweighted graphs (weights == NULL) reach the same picks without the serial sums: exact
 * class counts give W_i - u*T, decided against a proven rounding bound, with the serial
 * arithmetic only where the bound cannot decide; environment
 * DW_REPLAY_SERIAL=1 forces the serial arithmetic everywhere (a testing aid). */
int dw_walk_replay(const int64_t *row_ptr, const int32_t *col, const int32_t *col_sorted,
                   const double *weights, int64_t n_rows, const int32_t *starts, int64_t n_walks,
                   int32_t walk_length, int32_t method, double p, double q,
                   const double *uniforms, int32_t *out, int32_t *status, void *stream);

/* dw_walk_replay for DeepWalk on an unweighted graph over the edge-inline CSR `edges`
 * (dw_edges_inline_build): the same walks bit for bit (the exact picks of dw_walk_replay, with
 * the serial arithmetic where their bound cannot decide, DW_REPLAY_SERIAL honoured), one
 * dependent 16-B load per step. Replaces random_walk_generator.py:61-72 on unweighted graphs. */
int dw_walk_replay_inline(const int64_t *row_ptr, const int32_t *edges, int64_t n_rows,
                          const int32_t *starts, int64_t n_walks, int32_t walk_length,
                          const double *uniforms, int32_t *out, int32_t *status, void *stream);

/* dw_walk_replay for node2vec on an unweighted graph, over the per-row adjacency hash: the same
 * walks bit for bit. At a step t -> v it probes the shorter of the two lists — N(v)'s classes
 * from t's hash (adj_off / adj_hash), or N(t)'s members' positions in N(v) from v's hash and
 * adj_hpos (dw_adj_hash_positions) — then the exact picks' margin rule, with the serial
 * arithmetic (over col_sorted) where it cannot decide. edge_cn: NULL, or the per-edge class
 * counts of dw_edge_common_counts — a step then classifies N(v) only from its nearer end up to
 * the crossing (same walks). counters: NULL, or uint64[4]
 * (caller-zeroed) += {bytes, hash probes, list entries read, steps} — the realised traffic for
 * the walk roofline (bench.py). Replaces random_walk_generator.py:94-119 on unweighted graphs. */
int dw_walk_replay_indexed(const int64_t *row_ptr, const int32_t *col, const int32_t *col_sorted,
                           const int64_t *adj_off, const int32_t *adj_hash,
                           const int32_t *adj_hpos, const int32_t *hub_idx,
                           const uint32_t *hub_bits, int64_t hub_words,
                           const uint32_t *edge_cn, int64_t n_rows,
                           const int32_t *starts, int64_t n_walks, int32_t walk_length, double p,
                           double q, const double *uniforms, int32_t *out, int32_t *status,
                           uint64_t *counters, void *stream);

/* edge_cn uint32[n_edges] for every directed edge e = (t -> v = col[e]) of row t: bit 31 =
 * [t in N(v)], bits 0-30 = #{x in N(v) : x != t, x in N(t)} — the class counts (x == prev, x a
 * neighbour of prev) of a node2vec step t -> v (random_walk_generator.py:100-108), computed once
 * per graph over the shorter list against the other row: its neighbour bitmap (hub_idx /
 * hub_bits of dw_hub_bitmaps; NULL = none), else its adjacency hash (dw_adj_hash_build); both
 * directions of an undirected edge from one count (the reverse entry through adj_hpos,
 * dw_adj_hash_positions). The graph must be simple (no repeated neighbour in a row). */
int dw_edge_common_counts(const int64_t *row_ptr, const int32_t *col, const int64_t *adj_off,
                          const int32_t *adj_hash, const int32_t *adj_hpos,
                          const int32_t *hub_idx, const uint32_t *hub_bits, int64_t hub_words,
                          int64_t n_rows, int64_t n_edges, uint32_t *edge_cn, void *stream);

/* The node2vec position index, step 1: off int64[n_edges + 1] = exclusive prefix sums of the
 * common-neighbour counts C(e) (edge_cn bits 0-30; off[n_edges] = the index's entry count) and
 * byte_off int64[n_edges + 1] = those of the edges' byte sizes in the compact index: C(e)
 * entries of 2 B (uint16) when the target row col[e] has <= 65536 neighbours, else 4 B
 * (int32), rounded up to 4 B (byte_off[n_edges] = the index's size). tmp == NULL: *tmp_bytes =
 * the scans' scratch size, nothing launched. n_edges < 2^32. */
int dw_n2v_edge_offsets(const int64_t *row_ptr, const int32_t *col, const uint32_t *edge_cn,
                        int64_t n_edges, int64_t *off, int64_t *byte_off, void *tmp,
                        size_t *tmp_bytes, void *stream);

/* The node2vec position index, step 2, for the edges [e_begin, e_end) (random_walk_generator.py:
 * 100-108: at a step t -> v only the 1/p neighbour t and the 1/q neighbours N(t) ∩ N(v) weigh
 * other than 1): writes, at pos + byte_off[e], the positions in N(v) of the C(e) common
 * neighbours of edge e = (t -> v), ascending, as uint16 or int32 (dw_n2v_edge_offsets), and
 * pos_t[e] = the position of t in N(v) or -1. The chunk's entries are off[e_begin] - base ..
 * off[e_end] - base (base = off[e_begin], n_chunk_pos = off[e_end] - base < 2^31); scratch
 * int32[n_chunk_pos] holds the chunk's sorted positions. A caller bounds the scratch by cutting
 * the edges into chunks. Positions come from the shorter list as the counts do (same adjacency
 * index arguments as dw_edge_common_counts); a row whose positions disagree with its count sets
 * DW_S_BAD_CSR in *status. tmp == NULL: *tmp_bytes = the scratch size for n_chunk_pos entries
 * and e_end - e_begin edges. n_edges < 2^31. */
int dw_n2v_edge_index_build(const int64_t *row_ptr, const int32_t *col, const int64_t *adj_off,
                            const int32_t *adj_hash, const int32_t *adj_hpos,
                            const int32_t *hub_idx, const uint32_t *hub_bits, int64_t hub_words,
                            const uint32_t *edge_cn, const int64_t *off, const int64_t *byte_off,
                            int64_t n_rows, int64_t n_edges, int64_t e_begin, int64_t e_end,
                            int64_t base, int64_t n_chunk_pos, uint8_t *pos, int32_t *scratch,
                            int32_t *pos_t, void *tmp, size_t *tmp_bytes, int32_t *status,
                            void *stream);

/* The node2vec position index, step 3: rec int32[n_edges][8], the walker's 32-B edge records
 * {v, deg(v), row_ptr[v] lo, hi, byte_off[e] lo, hi, edge_cn[e], pos_t[e]}. */
int dw_n2v_edge_records(const int64_t *row_ptr, const int32_t *col, const uint32_t *edge_cn,
                        const int64_t *byte_off, const int32_t *pos_t, int64_t n_edges,
                        int32_t *rec, void *stream);

/* ---- deterministic accumulation (SURVEY.md §5 "race detection": run-to-run, eager / graph
 * and 1 / N-rank bit-identical tables) --------------------------------------------------------
 * Registers acc (int64[n_elems], zeroed by the caller) as the accumulator of the float gradient
 * buffer grad: every later SGNS launch whose g_in / g_out is grad adds each gradient term t as
 * round(t * 2^frac) into acc with integer atomics — sums independent of order and of how the
 * terms are split over waves, chunks or ranks — and converts the exact sums back into grad
 * (centre rows after pass 1, output rows in the records gather) unless flags has
 * DW_EXACT_DEFER: then acc keeps the centre sums for the caller to reduce across ranks and
 * convert (dw_fixed_to_float). The records (sorted) output path only; pooled (CBOW) inputs are
 * refused. frac: dw_exact_frac_bits(the launches' grad scale). Host-side registry, keyed by
 * the grad pointer (graph-captured launches keep the accumulator they were captured with). */
#define DW_EXACT_DEFER 1
/* (flags, a centre-table buffer of the one-GPU dense path) the dense Adam converts: pass 1 leaves
 * the centre sums in acc, and dw_adam_dense / dw_adam_dense_to on this buffer read each
 * gradient as fl(acc * 2^-frac) and clear acc (zero_grad) — one streaming pass instead of a
 * conversion pass after pass 1. */
#define DW_EXACT_ADAM 2

/* Row 0 of a lazy Adam history (dw_adam_rows): the box header's tag ("WDBX"). */
#define DW_HIST_BOX_TAG 0x58424457u
int dw_exact_register(const float *grad, int64_t *acc, int64_t n_elems, int32_t frac,
                      int32_t flags);
int dw_exact_unregister(const float *grad);
/* 32 + ceil(-log2 |scale|), clamped to [16, 62]: terms |coef| <= |scale| times entries below
 * 2^19 stay under 2^51, sums under 2^31 fit int64. */
int32_t dw_exact_frac_bits(double scale);
/* grad[i] = (accumulate ? grad[i] : 0) + fl(acc[i] * 2^-frac); acc[i] = 0 (i < n). */
int dw_fixed_to_float(int64_t *acc, float *grad, int64_t n, int32_t frac, int32_t accumulate,
                      void *stream);

/* dw_walk_replay_indexed's walks, bit for bit, over the position index (n2v_rec / n2v_pos of
 * dw_n2v_edge_index_build): one lane per walker, a step reads its edge's 32-B record and
 * binary-searches that edge's positions (log2 C loads), the pick by the margin rule; a pick the
 * margin cannot decide is made by the reference's own fp64 arithmetic (sum, normalise,
 * accumulate, bisect_right) replayed run by run over the position list, O(C + log n) in the
 * walker's lane. counters: NULL, or uint64[5] (caller-zeroed) += {bytes, serial picks, position
 * 2-B units read, steps, the searches' dependent 128-B line moves (a probe in the line of the
 * probe before it not counted)}. Replaces random_walk_generator.py:94-119 on unweighted graphs. */
int dw_walk_replay_positions(const int64_t *row_ptr, const int32_t *n2v_rec,
                             const uint8_t *n2v_pos, int64_t n_rows, const int32_t *starts,
                             int64_t n_walks, int32_t walk_length, double p, double q,
                             const double *uniforms, int32_t *out, int32_t *status,
                             uint64_t *counters, void *stream);

/* Neighbour bitmaps of hub rows for dw_walk_replay_indexed (hub_idx / hub_bits; NULL = none):
 * bits[k * hub_words + (x >> 5)] bit (x & 31) = x in N(hub_rows[k]); hub_words >=
 * ceil(n_rows / 32). A test of a neighbour of v against a hub prev too long for LDS is then one
 * 4-B load instead of a binary search of its sorted list. */
int dw_hub_bitmaps(const int64_t *row_ptr, const int32_t *col, int64_t n_rows,
                   const int32_t *hub_rows, int64_t n_hubs, int64_t hub_words, uint32_t *bits,
                   void *stream);

/* Fast walker (Philox4x32-10 keyed by (seed, walk_id0 + w, step, round/lane)); walks are a pure
 * function of (seed, global walk id), identical for any grid and any number of GPUs.
 *   DeepWalk: one lane per walker; uniform neighbour (unweighted) or alias table (weighted).
 *   node2vec: 8 lanes per walker; rejection rounds of 64 proposals x ~ w(v,x) (Philox counter
 *   field j = 0..63), accepted with alpha(prev,x)/alpha_max under the reference's rule
 *   (x==prev -> 1/p, prev in N(x) -> 1/q, else 1; random_walk_generator.py:101-108); the
 *   lowest accepting j wins — an exact draw from the reference's step law. Proposals are
 *   evaluated 8 at a time in j order; adjacency is tested only where the uniform leaves the
 *   outcome open.
 * prob_thr/alias: NULL for unweighted graphs. col_sorted: required for node2vec (8-ary search
 * of the sorted list). dw_walk_fast_indexed: the same walks (bit-identical) over derived
 * indexes — DeepWalk over the edge-inline CSR `edges` (dw_edges_inline_build; one dependent
 * load per step, walks stored 4 steps per 16-B store), node2vec with its adjacency tests in the
 * per-row hash (adj_off/adj_hash from dw_adj_hash_build; `col` for rows of degree <= 8). */
int dw_walk_fast(const int64_t *row_ptr, const int32_t *col, const int32_t *col_sorted,
                 const uint32_t *prob_thr, const int32_t *alias, int64_t n_rows,
                 const int32_t *starts, int64_t n_walks, int32_t walk_length, int32_t method,
                 double p, double q, uint64_t seed, uint64_t walk_id0, int32_t *out,
                 int32_t *status, void *stream);
int dw_walk_fast_indexed(const int64_t *row_ptr, const int32_t *col, const int32_t *edges,
                         const int64_t *adj_off, const int32_t *adj_hash,
                         const uint32_t *prob_thr, const int32_t *alias, int64_t n_rows,
                         const int32_t *starts, int64_t n_walks, int32_t walk_length,
                         int32_t method, double p, double q, uint64_t seed, uint64_t walk_id0,
                         int32_t *out, int32_t *status, void *stream);

/* dw_walk_fast_indexed's node2vec walks (the same walks, bit for bit) with the walker's realised
 * memory traffic counted, for the walk roofline (bench.py): counters[0..3] (uint64, caller-zeroed,
 * accumulated) += load + store bytes the walkers issued (row_ptr / adj_off pairs, proposal picks,
 * hash buckets or short-list scans, the output), steps, proposal blocks evaluated, adjacency
 * tests. A diagnostic launch: one wave-summed atomic per counter and wave. Replaces no reference
 * interface (the reference has no counters); its walks are Node2Vec.walk's law
 * (random_walk_generator.py:94-119). */
int dw_walk_fast_counted(const int64_t *row_ptr, const int32_t *col, const int64_t *adj_off,
                         const int32_t *adj_hash, const uint32_t *prob_thr, const int32_t *alias,
                         int64_t n_rows, const int32_t *starts, int64_t n_walks,
                         int32_t walk_length, double p, double q, uint64_t seed,
                         uint64_t walk_id0, int32_t *out, int32_t *status,
                         uint64_t *counters, void *stream);

/* node2vec with Philox draws over the per-edge position index (n2v_rec / n2v_pos from
 * dw_n2v_edge_index_build): one lane per walker, one 32-B edge record and log2 C dependent 2-B
 * (4-B for a hub target's list) position loads per step, no rejection rounds. The law is Node2Vec.walk's
 * (random_walk_generator.py:94-119, the reference's inverted q rule): step 1 picks
 * bounded32(r.x, deg) (:97, prev None), later steps the first neighbour i whose exact prefix
 * weight W_i = a_i/p + b_i + c_i/q exceeds U*T, U = 53 bits of (r.x, r.y), with the fp64
 * expressions of the exact replay's pick; Philox counter (walk id lo, hi, step << 8, 'NP').
 * Unweighted graphs (the index has no weights). counters: NULL, or uint64[4] += {load + store
 * bytes, steps, the searches' dependent 128-B line moves, position 2-B units read}. Reads
 * walk_id0 from a bound dw_step_scalars block. */
int dw_walk_fast_positions(const int64_t *row_ptr, const int32_t *n2v_rec, const uint8_t *n2v_pos,
                           int64_t n_rows, const int32_t *starts, int64_t n_walks,
                           int32_t walk_length, double p, double q, uint64_t seed,
                           uint64_t walk_id0, int32_t *out, int32_t *status, uint64_t *counters,
                           void *stream);

/* Edge-inline CSR for DeepWalk in dw_walk_fast_indexed: edges int32[nnz][4], entry e of row u =
 * {x = col[e], deg(x), row_ptr[x] low 32 bits, row_ptr[x] high 32 bits}. The pick of the next
 * node then also yields its row: one dependent load per walk step instead of two — the
 * `get_node_neighbors` + `random.choices` step of DeepWalk.walk (random_walk_generator.py:41-42,
 * 61-72) as one 16-B read. */
int dw_edges_inline_build(const int64_t *row_ptr, const int32_t *col, int64_t n_rows, int64_t nnz,
                          int32_t *edges, void *stream);

/* ---- SGNS (skip-gram negative sampling) ---------------------------------------------------------- */

/* Fused SGNS over walks: W2VCollateFunctional sg windows (torch_dataset.py:300-309) +
 * generate_noise_batch (sampling.py:7-21) + SkipGram.forward x2 (model.py:79-91) +
 * NegativeSamplingLoss (loss.py:14-22) + the closed-form backward of all of it
 * (clamp(sigmoid,1e-6) zero-gradient mask), accumulated into dense gradient tables.
 *   walks: int32[n_walks, L] vocabulary ids; centres are positions R..L-R-1 of every walk,
 *          centre b = w*(L-2R) + (i-R); contexts left-then-right.
 *   noise: int64[B', 2R, K] replayed negatives, or NULL = draw uniform [0,V) on device with
 *          Philox keyed by (seed, noise_offset + b, j*K + k).
 *   w_in/w_out: float32[V, d] (in/out embedding tables, row-major);
 *   g_in/g_out: float32[V, d] gradients, ACCUMULATED (+=);
 *   grad_scale: d(loss)/d(term) = 1/M, M = total centres*2R of the (global) batch.
 *   loss_acc: float64[4] accumulated (+=): sum positive-loss, sum negative-loss (summed over K),
 *             count(sigmoid(s)>=0.5), count(sigmoid(t)>=0.5)  (trainer.py:145-150).
 *   workspace: NULL -> output-table gradients scattered with float atomics;
 *              non-NULL (>= dw_sgns_workspace_bytes) -> atomic-free output-table path: one
 *              {row, centre, coef} record per output row, radix-sorted by row, then summed per
 *              row from gathered centre rows (stable order: g_out is reproducible run to run
 *              except at rows straddling two 512-record chunks). The centre-table gradient is
 *              one float-atomic row per centre in both modes. */
int dw_sgns_walks(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                  int32_t context_radius, int32_t neg_samples, int64_t vocab_size, int32_t dim,
                  const float *w_in, const float *w_out, float *g_in, float *g_out,
                  const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
                  double *loss_acc, int32_t *status, void *workspace, size_t workspace_bytes,
                  void *stream);

/* Two-phase form of dw_sgns_walks (same arguments, plus phase): phase 1 runs pass 1 — the
 * centre-table gradient g_in, the loss sums and the output-row records in the workspace —
 * and phase 2 sorts the records and accumulates g_out. A phase-2 call must follow the phase-1
 * call with identical arguments on the same stream; between the two, g_in is final and may be
 * read (the multi-GPU exchange starts its reduce-scatter there, overlapping phase 2). phase 0
 * is dw_sgns_walks. In atomic mode (workspace NULL) phase 1 does everything. */
int dw_sgns_walks_phase(int32_t phase, const int32_t *walks, int64_t n_walks,
                        int32_t walk_length, int32_t context_radius, int32_t neg_samples,
                        int64_t vocab_size, int32_t dim, const float *w_in, const float *w_out,
                        float *g_in, float *g_out, const int64_t *noise, uint64_t seed,
                        uint64_t noise_offset, float grad_scale, double *loss_acc,
                        int32_t *status, void *workspace, size_t workspace_bytes,
                        void *stream);

/* Phase 2 of dw_sgns_walks_phase in row pieces (N > 1: ShardedTables pipelines each piece's
 * output-table exchange behind the next piece's gather). Piece p covers output rows
 * [p * piece_rows, (p+1) * piece_rows); n_pieces * piece_rows >= vocab_size, n_pieces <= 1024.
 *   piece == -1: the records sort of the preceding phase-1 call and the record bounds of the
 *                pieces (in the workspace);
 *   piece in [0, n_pieces): g_out += the gradient of piece p's rows (complete when it returns
 *                in stream order; other rows untouched).
 * Calls -1, 0, ..., n_pieces-1 in order equal phase 2. Arguments as dw_sgns_walks_phase, same
 * workspace (a workspace holds one sorted batch at a time). */
int dw_sgns_walks_phase2_piece(int32_t piece, int32_t n_pieces, int64_t piece_rows,
                               const int32_t *walks, int64_t n_walks, int32_t walk_length,
                               int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                               int32_t dim, const float *w_in, float *g_out, int32_t *status,
                               void *workspace, size_t workspace_bytes, void *stream);

/* Phase 2 of dw_sgns_walks_phase fused with the output table's dense Adam step (one device):
 * the same records sort + gather, but every out row is updated in place with torch.optim.Adam
 * (single-tensor semantics, the scalars of dw_adam_dense) using its complete gradient —
 * rows wholly inside one gather chunk straight from registers, the rest (chunk-boundary rows,
 * rows without records: g = 0) from g_out. Equals phase 2 followed by dw_adam_dense(w_out,
 * g_out, m_out, v_out, ..., zero_grad = 1); g_out must be zero on entry and is left zero;
 * row_flags: vocab_size bytes, zero on entry, left zero. Arguments as dw_sgns_walks_phase
 * (g_in, noise, seed, loss_acc are not used by phase 2). */
int dw_sgns_walks_phase2_adam(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                              int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                              int32_t dim, const float *w_in, float *w_out, float *g_out,
                              float *m_out, float *v_out, uint8_t *row_flags,
                              float one_minus_beta1, float beta2, float one_minus_beta2,
                              float bias_correction2_sqrt, float neg_step_size, float eps,
                              float weight_decay, int32_t *status, void *workspace,
                              size_t workspace_bytes, void *stream);

/* Owner-computes form of the walks SGNS step for N > 1 (ShardedTables(mode='owner'), bench.py).
 * The output ("context") table is sharded by row owner: rank `owner` of `n_owners` holds only
 * rows o with o % n_owners == owner, as local row o / n_owners of w_out_local
 * (float32[local_rows, d], local_rows * n_owners >= vocab_size). Every rank passes the WHOLE
 * global batch of walks (walks are keyed by global id, so each rank forms them itself) and the
 * full, replicated in table; it computes only the output slots it owns, so no output-table
 * gradient or parameter ever crosses ranks. Replaces the reference's single-device step
 * (trainer.py:131-152 + the dense Adam of config_parser/core.py:43-53) at N > 1; summed over the
 * owners, the work is exactly dw_sgns_walks_phase's.
 * pass 1: g_in += the centre-table gradient of the owned slots (a PARTIAL sum: the caller
 *         reduces it across ranks), loss_acc += their loss terms, records kept in the
 *         workspace (>= dw_sgns_owner_workspace_bytes(n_walks*(L-2R), 2R, K, V, local_rows)),
 *         packed in a fixed order (deterministic).
 *         Needs dim a multiple of 64 (<= 512) and 2R(1+K) <= 64 (else DW_E_UNSUPPORTED).
 * pass 2: sorts the records by local row and accumulates the slice's gradient: with m_out
 *         non-NULL, the slice's torch.optim.Adam step is fused in exactly as in
 *         dw_sgns_walks_phase2_adam (g_out_local zero on entry and left zero, row_flags
 *         local_rows bytes); with m_out NULL, g_out_local += the gradient. With n_records
 *         non-NULL it reads the record count back to the host (ONE synchronisation of
 *         `stream`) into *n_records and sorts exactly that many; with n_records NULL there is
 *         no synchronisation: the sort runs over the bound n_walks*(L-2R)*2R(1+K) with the
 *         tail padded past every row and the gather limited on the device — the choice for
 *         n_owners = 1, where every slot is kept and the bound is the count. Same walk sizes
 *         and workspace as the pass-1 call. */
int dw_sgns_owner_workspace_bytes(int64_t n_centres, int32_t n_ctx, int32_t neg_samples,
                                  int64_t vocab_size, int64_t local_rows, size_t *bytes);
/* The owner form's centre order for a batch ahead of pass 1 (pass 1 with order_ready = 1 uses
 * it instead of building its own): the centres sorted by node (stable). touched (optional,
 * uint32[n_walks*(L-2R)]) receives the batch's distinct centre nodes in increasing order and
 * *n_touched (device int64) their count — the rows a step reads and updates in the in table
 * (OwnerLazyTables). Same workspace as the pass-1 / pass-2 calls that follow.
 * dw_sgns_owner_pass1's order_ready is a bit set: 1 = this order is ready (else pass 1 builds
 * it); 2 = the records are placed (dw_sgns_owner_out_catch_up ran with flags & 1 on this batch
 * and workspace): pass 1 writes each record straight into its row's segment, and
 * dw_sgns_owner_pass2_lazy (flags & 1) gathers them without a sort; 4 (with 2) = coefficients in:
 * dw_sgns_owner_out_rows already formed every record's coefficient and left each row it stepped
 * pending, its pre-step values in w_out_local — pass 1 forms the centre gradient alone (no loss
 * sums, no records written; loss_acc may be NULL); 8 (with 4) = the centres in walk order (no
 * node order is built or read: one atomic row per centre occurrence). */
int dw_sgns_owner_prepare(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                          int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                          int64_t local_rows, uint32_t *touched, int64_t *n_touched,
                          void *workspace, size_t workspace_bytes, void *stream);
int dw_sgns_owner_pass1(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                        int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                        int32_t dim, int32_t owner, int32_t n_owners, int64_t local_rows,
                        int32_t order_ready, const float *w_in, const float *w_out_local,
                        float *g_in,
                        const int64_t *noise, uint64_t seed, uint64_t noise_offset,
                        float grad_scale, double *loss_acc, int32_t *status, void *workspace,
                        size_t workspace_bytes, void *stream);
int dw_sgns_owner_pass2(int64_t n_walks, int32_t walk_length, int32_t context_radius,
                        int32_t neg_samples, int64_t local_rows, int32_t dim, const float *w_in,
                        float *w_out_local, float *g_out_local, float *m_out, float *v_out,
                        uint8_t *row_flags, float one_minus_beta1, float beta2,
                        float one_minus_beta2, float bias_correction2_sqrt, float neg_step_size,
                        float eps, float weight_decay, int32_t *status, void *workspace,
                        size_t workspace_bytes, int64_t *n_records, void *stream);

/* The lazy out slice's catch-up, before dw_sgns_owner_pass1 of the same batch: every owned
 * output row a slot references (contexts from the walks, negatives as pass 1 draws them) is
 * brought current to step - 1 (its deferred g = 0 steps replayed, hist as above), so pass 1 reads
 * the rows the dense update holds. claim int32 [local_rows] (zero-initialised, never reset): a
 * row is listed once per step, claimed via atomicMax(claim[row], step), when its last claim is
 * older than step - 1; rows_buf uint32 [min(local_rows, B' * 2R(1+K))] and n_rows (int64,
 * device) receive the list, which is then replayed. flags (a bit set):
 *   1 = place the records: counts uint32 [local_rows + 1] (zero-initialised; the placement
 *       scan clears it once read, so it is zero between steps) counts every row's slots, each
 *       slot's rank among them and the exclusive scan of the counts go to `workspace` (the owner
 *       form's, dw_sgns_owner_workspace_bytes), for dw_sgns_owner_pass1 (order_ready | 2) and
 *       dw_sgns_owner_pass2_lazy (flags | 1, the same counts): the records land grouped by row,
 *       no sort (the order of one row's records is the order the atomics resolved);
 *   2 = replay p only: m, v and last_step stay behind, and dw_sgns_owner_pass2_lazy (flags | 2)
 *       replays m and v (a multiply each per step) before the step — valid while every step has
 *       weight_decay 0;
 *   4 (with 1) = the rows-major step follows (dw_sgns_owner_out_rows): only the ranks and the
 *       scan — no claim, no list, no replay — then every slot is placed (its row and slot id in
 *       the workspace's records); claim and rows_buf are not touched.
 * 2R(1+K) <= 64, dim <= 512. */
int dw_sgns_owner_out_catch_up(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                               int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                               int32_t dim, int32_t owner, int32_t n_owners, int64_t local_rows,
                               const int64_t *noise, uint64_t seed, uint64_t noise_offset,
                               float *w_out_local, float *m_out, float *v_out,
                               int32_t *last_step, int32_t *claim, uint32_t *counts,
                               uint32_t *rows_buf, int64_t *n_rows, const float *hist,
                               int32_t step, int32_t flags, int32_t *status, void *workspace,
                               size_t workspace_bytes, void *stream);

/* dw_sgns_owner_pass2 with the out slice's Adam kept LAZY and exact (OwnerLazyTables, small
 * batches): a row no record touched is not read or written; its deferred g = 0 steps are
 * replayed (scalars hist[t], fp32 [steps][8] as for dw_adam_rows) right before its next update,
 * through the same adam_elem, so the slice equals the dense update bit for bit once flushed
 * (dw_adam_rows with rows = NULL). last_step int32 [local_rows]: the step each row is current
 * to; step: this step (>= 1). torch.optim.Adam semantics (config_parser/core.py:43-53).
 * flags: 1 = the records were placed (see dw_sgns_owner_out_catch_up; n_records NULL; counts:
 * its row counts, already cleared by its scan), 2 = the catch-up replayed p only (m, v are
 * replayed here), 4 = every step so far had the same betas (those replays use this step's). */
int dw_sgns_owner_pass2_lazy(int64_t n_walks, int32_t walk_length, int32_t context_radius,
                             int32_t neg_samples, int64_t local_rows, int32_t dim,
                             const float *w_in, float *w_out_local, float *g_out_local,
                             float *m_out, float *v_out, int32_t *last_step, const float *hist,
                             int32_t step, int32_t flags, uint32_t *counts, int32_t *status,
                             void *workspace, size_t workspace_bytes, int64_t *n_records,
                             void *stream);

/* The distinct centre nodes of a batch (the in rows one step touches), UNSORTED, for the lazy
 * in-table update on one rank (dw_sgns_owner_prepare gives them sorted, the order every rank
 * agrees on when N > 1): claim int32 [vocab_size] (zero-initialised, kept across steps) gets
 * claim[node] = step and the first claimer lists the node in touched (uint32 [>= B']);
 * n_touched (int64, device) their count. fresh / n_fresh (NULL = not wanted): the listed
 * nodes whose claim was below step - 1 — not centres of the step before, so nothing of that
 * step writes their rows (the pipelined step catches them up while step - 1 still runs). Reads
 * step from a bound dw_step_scalars block (relative form). flags: 0, or 1 = the counters are
 * already zero (not reset here: a caller that clears many steps' counters at once). Replaces
 * nothing in the reference (its optimizer steps every row). */
int dw_sgns_owner_touch_claim(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                              int32_t context_radius, int64_t vocab_size, int32_t *claim,
                              int32_t step, uint32_t *touched, int64_t *n_touched,
                              uint32_t *fresh, int64_t *n_fresh, int32_t flags, void *stream);

/* The rows-major lazy out step (OwnerLazyTables, one device; after dw_sgns_owner_out_catch_up
 * with flags 1 | 4 on the same batch and workspace, before dw_sgns_owner_pass1 with order_ready
 * 1 | 2 | 4): each owned out row the batch touches is read once and written once — its deferred
 * g = 0 steps replayed (hist, as for dw_adam_rows), the logits of its records against their
 * centre rows, the coefficients and loss sums (loss_acc float64[4] as for dw_sgns_walks), its
 * gradient and the Adam step `step` — the same arithmetic as the catch-up / pass 1 /
 * dw_sgns_owner_pass2_lazy sequence. Leaves each record's coefficient in the placed records
 * and every row it steps PENDING for dw_sgns_owner_pass1's centre gradient: exp_avg and
 * exp_avg_sq at `step`, the parameter row still at step - 1 (what the centre gradient reads),
 * pending[row] = 1 (uint8 [local_rows], zero-initialised by the caller). The parameter half of
 * a pending row's step (torch Adam's p update from its m and v, the same operations) is applied
 * when the row is next replayed — by the next rows-major step, or by dw_adam_rows given the same
 * `pending` (the flush before the table is read whole). counts: the catch-up's (already cleared
 * by its placement scan; not written here). dim in {64, 128, 256, 512}, 2R(1+K) <= 64; the
 * deterministic mode (g_out registered) sums each row's terms as integers. */
int dw_sgns_owner_out_rows(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                           int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                           int32_t dim, int32_t owner, int32_t n_owners, int64_t local_rows,
                           const int64_t *noise, uint64_t seed, uint64_t noise_offset,
                           float grad_scale, const float *w_in, float *w_out_local,
                           float *g_out_local, float *m_out, float *v_out, int32_t *last_step,
                           uint32_t *counts, uint8_t *pending, const float *hist,
                           int32_t step, double *loss_acc, int32_t *status,
                           void *workspace, size_t workspace_bytes, void *stream);

/* Same computation over explicit pairs (the reference's collate output):
 * inputs int64[B], targets int64[B, C], noise int64[B, C, K] or NULL (Philox as above). */
int dw_sgns_pairs(const int64_t *inputs, const int64_t *targets, int64_t batch, int32_t n_ctx,
                  int32_t neg_samples, int64_t vocab_size, int32_t dim,
                  const float *w_in, const float *w_out, float *g_in, float *g_out,
                  const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
                  double *loss_acc, int32_t *status, void *workspace, size_t workspace_bytes,
                  void *stream);

/* Pooled-input (CBOW) form of dw_sgns_pairs (model.py:94-110 CBOW.forward + loss.py:14-22 +
 * trainer.py:131-152): the input vector of sample b is the mean of w_in rows inputs[b, 0..n_in)
 * (torch.mean over dim 1); targets int64 [batch, n_ctx] are the positive output rows and the
 * noise [batch, n_ctx, neg_samples] (or device Philox, NULL) the negatives. Each of the n_in
 * input rows receives 1/n_in of the input-vector gradient (mean backward). n_in = 1 computes
 * what dw_sgns_pairs computes. Always the atomic output-table scatter (text-corpus batches). */
int dw_sgns_pooled_pairs(const int64_t *inputs, int32_t n_in, const int64_t *targets,
                         int64_t batch, int32_t n_ctx, int32_t neg_samples, int64_t vocab_size,
                         int32_t dim, const float *w_in, const float *w_out, float *g_in,
                         float *g_out, const int64_t *noise, uint64_t seed,
                         uint64_t noise_offset, float grad_scale, double *loss_acc,
                         int32_t *status, void *stream);

/* The device negatives dw_sgns_* draw when noise == NULL, written out: noise[(b*n_ctx + j)*K + k]
 * for b < batch (centre counter noise_offset + b). Replaces generate_noise_batch
 * (utils/sampling.py:7-21) where the ids must exist before the step (max_norm renormalisation).*/
int dw_sgns_noise(int64_t batch, int32_t n_ctx, int32_t neg_samples, int64_t vocab_size,
                  uint64_t seed, uint64_t noise_offset, int64_t *noise, void *stream);

/* nn.Embedding(max_norm=...) lookup side effect (model.py:24-25 with max_norm set; torch
 * embedding_renorm_): every DISTINCT row among ids[0..n_ids) whose L2 norm exceeds max_norm is
 * scaled by max_norm / (norm + 1e-7), in place. Ids are deduplicated on the device (radix sort
 * in the caller's workspace, >= dw_embedding_renorm_workspace_bytes). Out-of-range ids set
 * DW_S_BAD_INDEX and are skipped. */
int dw_embedding_renorm_workspace_bytes(int64_t n_ids, int64_t vocab_size, size_t *bytes);
int dw_embedding_renorm(float *weight, int64_t vocab_size, int32_t dim, const int64_t *ids,
                        int64_t n_ids, double max_norm, void *workspace, size_t workspace_bytes,
                        int32_t *status, void *stream);

/* Bytes of device workspace the records path needs for n_centres centres with n_ctx contexts
 * and neg_samples negatives each over a vocabulary of vocab_size rows. */
int dw_sgns_workspace_bytes(int64_t n_centres, int32_t n_ctx, int32_t neg_samples,
                            int64_t vocab_size, size_t *bytes);

/* Profiling aid (bench.py): enable != 0 starts (and resets) per-phase HIP-event timing of every
 * later dw_sgns_walks / dw_sgns_pairs call on this process; enable == 0 stops it.
 * dw_sgns_phase_ms waits for the last recorded call and returns the mean milliseconds of
 * ms[0] pass 1 (k_sgns*: logits, loss, centre gradients, records), ms[1] the radix sort of the
 * records, ms[2] pass 2 (k_rec_gather: output-table gradients) over *n_calls calls (ms[1],
 * ms[2] are 0 in atomic mode). No reference counterpart (measurement only). */
int dw_sgns_timing(int32_t enable);
int dw_sgns_phase_ms(double *ms, int64_t *n_calls);

/* CBOW.forward(inputs, outputs, proba) (model.py:98-110): logits[b, n] =
 * <mean_p w_in[inputs[b, p]], w_out[outputs[b, n]]>, p < n_in; dw_skipgram_logits is n_in = 1.
 * The backward adds dlogits[b,n] * pooled_b into g_out[outputs[b,n]] and (sum_n dlogits[b,n] *
 * w_out[outputs[b,n]]) / n_in into each g_in[inputs[b, p]]. */
int dw_pooled_logits(const int64_t *inputs, int32_t n_in, const int64_t *outputs,
                     int64_t batch, int32_t n_out, int64_t vocab_size, int32_t dim,
                     const float *w_in, const float *w_out, int32_t proba, float *logits,
                     int32_t *status, void *stream);
int dw_pooled_logits_backward(const int64_t *inputs, int32_t n_in, const int64_t *outputs,
                              int64_t batch, int32_t n_out, int64_t vocab_size, int32_t dim,
                              const float *w_in, const float *w_out, const float *dlogits,
                              float *g_in, float *g_out, int32_t *status, void *stream);

/* SkipGram.forward(inputs, outputs, proba) (model.py:79-91): logits[b, n] =
 * <w_in[inputs[b]], w_out[outputs[b, n]]>, sigmoid applied when proba != 0. */
int dw_skipgram_logits(const int64_t *inputs, const int64_t *outputs, int64_t batch,
                       int32_t n_out, int64_t vocab_size, int32_t dim, const float *w_in,
                       const float *w_out, int32_t proba, float *logits, int32_t *status,
                       void *stream);

/* Backward of dw_skipgram_logits (proba == 0): g_in[inputs[b]] += sum_n dlogits[b,n] w_out[..],
 * g_out[outputs[b,n]] += dlogits[b,n] w_in[inputs[b]] (the embedding_dense_backward of
 * model.py:85-88 under autograd). */
int dw_skipgram_logits_backward(const int64_t *inputs, const int64_t *outputs, int64_t batch,
                                int32_t n_out, int64_t vocab_size, int32_t dim,
                                const float *w_in, const float *w_out, const float *dlogits,
                                float *g_in, float *g_out, int32_t *status, void *stream);

/* Dense Adam step, torch.optim.Adam single-tensor semantics (torch/optim/adam.py:_single_tensor_adam,
 * amsgrad=False), configured by config_parser/core.py:43-53. Host computes the per-step scalars
 * in float64 exactly as torch does; the kernel runs the fp32 tensor ops:
 *   m = lerp(m, g, one_minus_beta1); v = v*beta2 + one_minus_beta2*g*g;
 *   denom = sqrt(v)/bias_correction2_sqrt + eps; p += neg_step_size * m/denom;
 * weight_decay != 0 adds weight_decay*p to g first (L2, non-decoupled).
 * zero_grad != 0 also writes g = 0 (fuses optimizer.zero_grad into the same HBM pass). */
int dw_adam_dense(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n_elem,
                  float one_minus_beta1, float beta2, float one_minus_beta2,
                  float bias_correction2_sqrt, float neg_step_size, float eps,
                  float weight_decay, int32_t zero_grad, void *stream);

/* dw_adam_dense reading the parameters from param_src and writing them to param_dst (the other
 * buffer of a double-buffered table, so readers of the current values can run concurrently);
 * param_src == param_dst is dw_adam_dense. max_blocks > 0 caps the grid (256-thread blocks,
 * grid-stride): a concurrent kernel on another stream keeps the rest of the CUs; <= 0 = the
 * full grid. */
int dw_adam_dense_to(const float *param_src, float *param_dst, float *grad, float *exp_avg,
                     float *exp_avg_sq, int64_t n_elem, float one_minus_beta1, float beta2,
                     float one_minus_beta2, float bias_correction2_sqrt, float neg_step_size,
                     float eps, float weight_decay, int32_t zero_grad, int64_t max_blocks,
                     void *stream);

/* Scale a float32 buffer in place: x *= alpha * (*alpha_dev) (alpha_dev NULL -> 1). Used by the
 * autograd path to apply the device-resident grad_output without a host synchronisation. */
/* Lazy exact Adam over selected rows (OwnerLazyTables, the touched-row in-table exchange;
 * torch.optim.Adam single-tensor semantics as dw_adam_dense). A row's update with g = 0 is a
 * fixed recurrence, so rows no batch touched are brought up to date later by replaying each
 * missed step through the same per-element arithmetic: the result is bit-identical to the
 * dense update every step.
 *   rows: uint32 row ids (NULL = rows 0 .. n_rows_max-1); n_rows_dev: device int64 count
 *         (NULL = n_rows_max; clamped to n_rows_max); ids >= n_table_rows are skipped;
 *   last_step: int32[n_table_rows], the step each row's (param, exp_avg, exp_avg_sq) are
 *         current to; updated;
 *   hist: float32[(step+1) * 8]: row s = Adam step s's scalars in dw_adam_dense's order
 *         (1-beta1, beta2, 1-beta2, sqrt(bias_correction2), -lr/bias_correction1, eps,
 *         weight_decay), then fp32 1 / sqrt(bias_correction2) correctly rounded (0 = not given:
 *         the kernels divide; given, they take three operations for the same quotient);
 *         row 0 (no step) may hold the box header: [0] = the bits of DW_HIST_BOX_TAG, [1] = the
 *         bits of an int32 step b such that every row s >= b up to the last one a launch reads
 *         has weight_decay +0, the reciprocal, eps in [2^-27, 1], sqrt(bias_correction2) in
 *         [2^-10, 1] and 1-beta1, beta2 in [0, 1]: the g = 0 replays of rows last current at
 *         b - 1 or later then run sqrt and the division without range scaling (the same bits,
 *         fewer operations); [2] = F, [3] = eps of those rows: with every box row's eps equal to
 *         it, (1 - beta1)(1 + 2^-20) <= sqrt(beta2) and |nstep| <= F, a replay whose parameter
 *         can provably no longer move (|m| F / max(RN(sqrt(v)), eps) below |p| 2^-26) steps m
 *         and v alone for the rest of the run (the same bits; F = +inf: never); [4] = 1-beta1,
 *         [5] = beta2 when every box row has those same values (the frozen steps then take them
 *         from here, not from each row; NaN = the betas vary); any other row 0 = no step in the
 *         box;
 *   grad_rows NULL: replay every listed row up to `step` (g = 0);
 *   grad_rows float32[n_rows_max, dim]: replay up to step - 1, then apply `step` with row i's
 *         gradient grad_rows[i];
 *   grad_by_row (with grad_rows): grad_rows is the table's dense gradient [n_table_rows, dim]
 *         and row r steps with grad_rows[r], which is cleared as it is read (one rank's touched
 *         rows: no gather);
 *   pending: NULL, or uint8 [n_table_rows] (dw_sgns_owner_out_rows): a listed row marked there
 *         first gets the parameter half of step last_step[r], and its mark is cleared; only
 *         with grad_rows NULL (a settle-and-replay: a gradient step on a pending row current to
 *         `step` would apply that step twice) — DW_E_INVALID_ARG otherwise. */
int dw_adam_rows(float *param, float *exp_avg, float *exp_avg_sq, int32_t *last_step,
                 uint8_t *pending, int64_t n_table_rows, int32_t dim, const uint32_t *rows,
                 const int64_t *n_rows_dev, int64_t n_rows_max, float *grad_rows,
                 int32_t grad_by_row, const float *hist, int32_t step, void *stream);

/* out[i] = table[rows[i]] for i < min(*n_rows_dev, n_rows_max) (float32 rows of dim); with
 * zero_source the table rows are cleared in the same pass (the touched rows of the in-table
 * gradient, gathered for the all-reduce). */
int dw_rows_gather(float *table, int64_t n_table_rows, int32_t dim, const uint32_t *rows,
                   const int64_t *n_rows_dev, int64_t n_rows_max, float *out,
                   int32_t zero_source, void *stream);

int dw_scale(float *x, int64_t n_elem, float alpha, const float *alpha_dev, void *stream);

/* ---- step scalars in device memory (HIP-graph replay of a training step) ------------------------
 * A small-batch training step is a few dozen microseconds of kernels; launched one by one from
 * the host it is launch-bound. To replay a captured step (hipGraph), the values that change from
 * step to step live in device memory instead of kernel arguments: while a dw_step_scalars block
 * is BOUND (dw_step_scalars_bind, per host thread), every launch of
 *   dw_walk_fast / dw_walk_fast_indexed / dw_walk_fast_positions   reads walk_id0 from it,
 *   dw_sgns_walks_phase (pass 1)          reads noise_offset from it,
 *   dw_adam_dense(_to), dw_sgns_walks_phase2_adam   read the Adam scalars adam[0..6],
 * and ignores the corresponding host arguments. dw_step_scalars_advance, the last node of a
 * captured step, moves the block to the next step. Nothing else changes: the kernels and their
 * results are those of the eager launches (the bench and tests compare the two). Replaces no
 * reference interface: it is how trainer.py:131-152's per-batch step is replayed on the device. */
typedef struct dw_step_scalars {
    uint64_t walk_id0;      /* global walk id of the step's first walk */
    uint64_t noise_offset;  /* centre counter of the step's device negatives */
    int64_t step;           /* the Adam step this step applies (1-based) */
    float adam[8];          /* its scalars, dw_adam_dense order, then RN(1/bias_correction2_sqrt) or 0 (a dw_adam_rows hist row) */
} dw_step_scalars;

/* Bind (dev != NULL) or unbind (NULL) a device dw_step_scalars for the launches this host
 * thread makes next. */
int dw_step_scalars_bind(const dw_step_scalars *dev);

/* As dw_step_scalars_bind, and the launches' Adam step numbers become relative to the block:
 * dw_adam_rows, dw_sgns_owner_out_catch_up and dw_sgns_owner_pass2_lazy then apply
 * dev->step + (step - host_step), read on the device, where `step` is their argument (the lazy
 * exact Adam of a captured one-GPU owner step: word2vec/graphed.py GraphedOwnerStep). Those
 * three refuse (DW_E_INVALID_ARG) a block bound without its host step. */
int dw_step_scalars_bind_at(const dw_step_scalars *dev, int64_t host_step);

/* walk_id0 += walks_per_step, noise_offset += centres_per_step, step += 1, adam = hist[step]
 * (hist: float32[hist_rows][8]; a step beyond hist_rows sets DW_S_BAD_INDEX in status and
 * leaves adam unchanged); then, with epoch_starts != NULL, the new step's start nodes into
 * starts_out exactly as dw_step_starts (one launch for both). */
int dw_step_scalars_advance(dw_step_scalars *dev, const float *hist, int64_t hist_rows,
                            uint64_t walks_per_step, uint64_t centres_per_step, int32_t *status,
                            const int32_t *epoch_starts, int64_t n_epoch, int32_t *starts_out,
                            int64_t n, void *stream);

/* Several steps in one launch (a graph that replays n_steps steps): steps[j] = *base advanced j
 * times as dw_step_scalars_advance would (j = 0 .. n_steps-1), then *base advanced n_steps
 * times; with epoch_starts != NULL, starts_out[k] = epoch_starts[(steps[0].walk_id0 + k) mod
 * n_epoch] for k < n (the start nodes of all n_steps steps' walks). Binding &steps[j] for step
 * j's launches replaces the n_steps advance launches of a captured multi-step graph. */
int dw_step_scalars_expand(dw_step_scalars *base, dw_step_scalars *steps, int64_t n_steps,
                           const float *hist, int64_t hist_rows, uint64_t walks_per_step,
                           uint64_t centres_per_step, int32_t *status,
                           const int32_t *epoch_starts, int64_t n_epoch, int32_t *starts_out,
                           int64_t n, void *stream);

/* starts_out[k] = epoch_starts[(dev->walk_id0 + k) mod n_epoch] for k < n: the start nodes of
 * a step's walks when walk w of the epoch starts at epoch_starts[w] (RandomWalkDataset's
 * `_get_current_node`, datasets.py:69-76, with the walk ids of the epoch). */
int dw_step_starts(const dw_step_scalars *dev, const int32_t *epoch_starts, int64_t n_epoch,
                   int32_t *starts_out, int64_t n, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* DW_HIP_H */
