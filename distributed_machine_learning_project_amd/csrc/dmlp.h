// dmlp.h — C ABI of libdmlp.so, the native core of the MI355X k-NN framework.
//
// Everything the reference computes in its hot loops is exposed
// here as plain C entry points so that (a) Python binds them with ctypes (no torch headers,
// no hipify, no JIT) and (b) the standalone MPI/RCCL `knn_engine` binary links the very same
// code.  All GPU entry points are asynchronous on the given HIP stream and return 0 on a
// successful launch, or a negative error code.  CPU entry points are synchronous.
//
// Numerical contract (reference common.cpp:57-79, engine.cpp:12-18):
//   dist(q,x) = sum_{a=0}^{A-1} (q_a - x_a)^2, IEEE double, left to right, no FMA;
//   order     = (dist ascending, id descending);
//   vote      = max count, ties -> larger label; empty -> -1;
//   checksum  = FNV-1a-64: h ^= (u64)label; h *= P; for id in order: h ^= (u64)(id+1); h *= P.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---------------------------------------------------------------- device: data preparation (K1)
// mu[A] = mean of the first min(N, 4096) rows (centering offset for the screen; any value is
// correct, a good one only tightens the screen).
int dmlp_center(const double* X, int64_t N, int A, double* mu, void* stream);
// The exact path's fp64 MFMA screen (screen_f64.hip) + exact group re-rank: k <= 64, A <= 32,
// results bit-identical to dmlp_exact_topk; overflowing queries get status[q] = 1 (nothing
// written) and are counted into *ovf_count (device).  ws: dmlp_exact_f64_bytes bytes.
int dmlp_exact_f64_amax(void);
int dmlp_exact_f64_kmax(void);
int64_t dmlp_exact_f64_bytes(int64_t N, int A, int nq, int kmax);
int dmlp_exact_f64(const double* X, int64_t N, int A, const double* Qx, const int* qidx,
                   const int* qk, int nq, int kmax, double* out_d, int* out_i, int kstride,
                   int* status, int* ovf_count, void* ws, int64_t ws_bytes, void* stream);
int dmlp_refine_groups_exact(int cap, const int* cand_ids, const int* cand_cnt, const float* cand_h,
                             int S, int64_t tiles_per_slice, const double* X, int A,
                             const double* Qx, int64_t n_points, const int* qidx, const int* qk,
                             int nq, double* out_d, int* out_i, int kstride, int* status,
                             int* ovf_count, void* stream);

// X [N][A] fp64 -> fragment-native bf16 hi/lo tiles (64 points x 32*KT attrs per tile),
// xinit[n_tiles*64] = -(|x-mu|^2)/2 (fp32; -inf for padding), xnmax_bits = max |x-mu|^2 (fp32
// bits), bad |= 1 if any value is non-finite or too large for the bf16x3 screen.
int dmlp_prep_data(const double* X, int64_t N, int A, const double* mu, int KT, void* xfrag,
                   float* xinit, unsigned* xnmax_bits, unsigned* bad, void* stream);

// Qx [Q][A] fp64 -> qhi/qlo [Q][32*KT] bf16, qn[Q] = |q-mu|^2 (fp32).
int dmlp_prep_queries(const double* Qx, int64_t Q, int A, const double* mu, int KT, void* qhi,
                      void* qlo, float* qn, unsigned* bad, void* stream);

// host_prep.cpp: the screen's query operands rendered on the host (persistent thread pool) —
// mu over the first min(N, 4096) rows like dmlp_center; qhi [Q][KT*32] fp16 bits, qn [Q] fp32.
// dmlp_cpu_prep_queries returns 1 if some |q - mu| is outside the screen's range.
int dmlp_host_threads(void);
// fn(ctx, part, parts) on the render pool's workers and the caller (host_prep.cpp)
void dmlp_host_pool_run(void (*fn)(void*, int, int), void* ctx);
void dmlp_cpu_center(const double* X, int64_t N, int A, double* mu);
int dmlp_cpu_prep_queries(const double* Qx, int64_t Q, int A, const double* mu, int KT,
                          uint16_t* qhi, float* qn);
// The dataset's single-term operands: the hi-only tile image (hl = 1 in dmlp_screen_x1 /
// dmlp_refine_groups), xinit and the max norm bits.  Returns 1 if outside the screen's range.
int dmlp_cpu_prep_data(const double* X, int64_t N, int A, const double* mu, int KT,
                       uint16_t* xhi, float* xinit, unsigned* xnmax_bits);
// Async device->host copy on `stream` (dst: page-locked or host-registered memory).
// Row-pointer-table variants of the host render (the engine.h drop-in reads the harness's
// per-point attribute vectors in place): centre, screen operands + H2D, lossless int32 pack,
// fp64 pack.
void dmlp_cpu_center_rows(const double* const* rows, int64_t N, int A, double* mu);
int dmlp_cpu_prep_queries_rows(const double* const* rows, int64_t Q, int A, const double* mu,
                               int KT, uint16_t* qhi, float* qn);
int dmlp_cpu_prep_data_tiles_rows(const double* const* rows, int64_t N, int A, const double* mu,
                                  int KT, int64_t t0, int64_t t1, uint16_t* xhi, float* xinit,
                                  float* nmax);
int dmlp_host_ops_h2d_tiles_rows(const double* const* Xr, int64_t N, int64_t t0, int64_t t1,
                                 const double* const* Qr, int64_t Q, int A, const double* mu,
                                 int KT, uint16_t* xhi_h, float* xin_h, unsigned* xnm_h,
                                 uint16_t* qhi_h, float* qn_h, void* xhi_d, void* xin_d,
                                 void* xnm_d, void* qhi_d, void* qn_d, int chunks, void* stream);
int dmlp_cpu_rows_i32_rows(const double* const* rows, int64_t nrows, int A, int32_t* dst);
void dmlp_cpu_gather_rows(const double* const* rows, int64_t nrows, int A, double* dst);
// Lossless 6-decimal transfer: int32 m with x == fl(m / 1e6) bit for bit (0 = every value
// passed, 1 = ship fp64), and the device reconstruction of the fp64 rows.
int dmlp_cpu_rows_i32(const double* src, int64_t n, int32_t* dst);
int dmlp_rows_from_i32(const int* src, int64_t n, double* dst, void* stream);
// The single-term screen's fp16 operands rendered on the device from rows that landed (prep.hip
// k_render; bit for bit the host render of host_prep.cpp): src32 int32 m (x = m / 1e6, also
// written to dst64 as the fp64 rows) or src64 fp64, rows [r0, r0 + n) of the whole array.  mode 0:
// dataset (n, r0 multiples of 64; rows >= nvalid pad) -> tile image img, xinit xq, point-major
// copy xrow (nullable), rounded-up max norm -> atomicMax(*nmax); mode 1: queries -> qhi img
// [row][KT 32], qn xq.  |x - mu| out of the fp16 range sets *bad (nullable).  done / rdy
// (nullable, *done zeroed by the caller): the last workgroup publishes *rdy = 1.
int dmlp_render_rows(int KT, int A, const int* src32, const double* src64, int64_t r0, int64_t n,
                     int64_t nvalid, const double* mu, double* dst64, int mode, void* img,
                     float* xq, void* xrow, unsigned* nmax, unsigned* bad, unsigned* done,
                     unsigned* rdy, void* stream);
int dmlp_d2h_async(void* dst, const void* src, int64_t bytes, void* stream);
int dmlp_cpu_prep_data_tiles(const double* X, int64_t N, int A, const double* mu, int KT,
                             int64_t t0, int64_t t1, uint16_t* xhi, float* xinit, float* nmax);
// Both operand sets rendered in `chunks` slices each (data first), every slice copied to the
// device on `stream` (hipMemcpyAsync from the page-locked *_h buffers) as soon as it is ready,
// so the host conversion overlaps PCIe.  Returns 0, or | 1 (data) / | 2 (queries) when some
// value is outside the screen's range (then those device operands are not usable).
int dmlp_host_ops_h2d(const double* X, int64_t N, const double* Qx, int64_t Q, int A,
                      const double* mu, int KT, uint16_t* xhi_h, float* xin_h, unsigned* xnm_h,
                      uint16_t* qhi_h, float* qn_h, void* xhi_d, void* xin_d, void* xnm_d,
                      void* qhi_d, void* qn_d, int chunks, void* stream);
// Same, the dataset part restricted to tiles [t0, t1) (device image pointers at tile t0's slot;
// *xnm = +inf when the range is outside the screen's range): the per-rank shard of a sharded render.
int dmlp_host_ops_h2d_tiles(const double* X, int64_t N, int64_t t0, int64_t t1, const double* Qx,
                            int64_t Q, int A, const double* mu, int KT, uint16_t* xhi_h,
                            float* xin_h, unsigned* xnm_h, uint16_t* qhi_h, float* qn_h,
                            void* xhi_d, void* xin_d, void* xnm_d, void* qhi_d, void* qn_d,
                            int chunks, void* stream);

// ---------------------------------------------------------------- device: screen (K2+K3, fused)
// bf16x3 MFMA screen + per-query streaming threshold + candidate compaction.  Queries are the
// class list qidx[0..nq); data is split into S slices.  Output: for class position p and slice s,
// cand_cnt[p*S+s] candidates (or -1 on overflow) stored at cand_ids[(p*S+s)*cap ...].
// cap in {128, 256}; the k of every query in the list must be <= dmlp_screen_kmax(cap).
int dmlp_screen_kmax(int cap);
// xnmax_bits / bad are the device words written by dmlp_prep_data (no host round trip).
int dmlp_screen(int KT, int cap, const void* xfrag, const float* xinit, int64_t n_tiles,
                const void* qhi, const void* qlo, const float* qn, const int* qidx, const int* qk,
                int nq, const unsigned* xnmax_bits, const unsigned* bad, float eps_rel, int S,
                int* cand_ids, int* cand_cnt, void* stream);
int dmlp_screen_lds_bytes(int KT, int cap);
int dmlp_screen_waves(int KT, int cap);
// hl = 2: the call above; hl = 1: the single-term form on the host's fp16 image and fp16 query
// fragments (dmlp_host_ops_h2d's operands; qlo / eps_rel unused, A selects the bound).
int dmlp_screen_hl(int KT, int cap, int hl, int A, const void* xfrag, const float* xinit,
                   int64_t n_tiles, const void* qhi, const void* qlo, const float* qn,
                   const int* qidx, const int* qk, int nq, const unsigned* xnmax_bits,
                   const unsigned* bad, float eps_rel, int S, int* cand_ids, int* cand_cnt,
                   void* stream);
int dmlp_screen_lds_bytes_hl(int KT, int cap, int hl);
int dmlp_screen_waves_hl(int KT, int cap, int hl);

// Barrier-free streaming screen (screen_stream.hip) for k <= dmlp_screen_stream_kmax() and
// KT <= 2: dmlp_screen_stream_qw(KT) queries per workgroup (0 = unsupported KT); kmax = the
// largest k in the query list; candidate ids per (query, slice) = dmlp_screen_stream_cap(kmax);
// same output contract as dmlp_screen.
int dmlp_screen_stream_qw(int KT);
int dmlp_screen_stream_cap(int kmax);
int dmlp_screen_stream_kmax(void);
int dmlp_screen_stream_waves_per_cu(int kmax);
int dmlp_screen_stream(int KT, const void* xfrag, const float* xinit, int64_t n_tiles,
                       const void* qhi, const void* qlo, const float* qn, const int* qidx,
                       const int* qk, int nq, int kmax, const unsigned* xnmax_bits,
                       const unsigned* bad, float eps_rel, int S, int* cand_ids, int* cand_cnt,
                       void* stream);
// 32-attribute fragments per row of the screen images for A attributes: A <= 256 rounds up to
// 1, 2, 4 or 8 (the single-term screen's variants; the zero padding costs MFMA work only), wider
// rows take ceil(A / 32) (exact path only).
static inline int dmlp_screen_kt(int A) {
  const int kt = A > 32 ? (A + 31) / 32 : 1;
  return kt > 8 ? kt : (kt <= 1 ? 1 : kt <= 2 ? 2 : kt <= 4 ? 4 : 8);
}
// Single-term bf16 screen (screen_x1.hip) for k <= dmlp_screen_x1_kmax() and KT in {1,2,4,8}: 64 queries
// per workgroup; A and the real point count are needed for the error bound and to drop padding
// rows; S >= dmlp_screen_x1_min_slices.  Output per (query, slice): up to dmlp_screen_x1_cap(kmax)
// 4-row group entries (ordered 16-bit key << 16 | slice-relative group index; count -1 =
// overflow) and cand_h[2] = {slice threshold, query eps} — consumed by dmlp_refine_groups.
int dmlp_screen_x1_kmax(void);
int dmlp_screen_x1_qw(int KT);
int dmlp_screen_x1_cols(int KT, int kmax);
int dmlp_screen_x1_cap(int kmax);  // (KT 1's; the image of KT fragments per step: _kt)
int dmlp_screen_x1_cap_kt(int KT, int kmax);
// rows per group entry of that screen's lists: 8 for kmax <= 16 (hit test and append once per two
// MFMA steps on the 8-row max: rows 4 kg .. 4 kg + 3 of steps 2p and 2p + 1, entry index 4 p + kg),
// else 4 (consecutive rows, entry index = row / 4); the refines expand each entry to its rows
int dmlp_screen_x1_group_rows(int kmax);
int dmlp_screen_x1_group_rows_kt(int KT, int kmax);
int dmlp_screen_x1_waves_per_cu(int kmax);
int dmlp_screen_x1_waves_per_cu_kt(int KT, int kmax);  // A > 64: one wave per SIMD
int64_t dmlp_screen_x1_min_slices(int64_t n_tiles);
void dmlp_screen_x1_bound(int A, float* r1, float* r2);
// eps(q) = r1 |q'| max|x'| + r2 max|x'|^2 + r3 (|q'| + max|x'| + 2^-15) for image kind hl
// (1: fp16 hi-only, 2: bf16 hi/lo)
void dmlp_screen_x1_bound2(int A, int hl, float* r1, float* r2, float* r3);
// hl: fragment halves per (step, kt) in xfrag — 2 for prep.hip's bf16 hi/lo image, 1 for the fp16
// hi-only image of dmlp_cpu_prep_data (the query fragments qhi must be of the same element type:
// fp16 from dmlp_cpu_prep_queries with hl = 1, bf16 from dmlp_prep_queries with hl = 2; same for
// dmlp_refine_groups).
int dmlp_screen_x1(int KT, int hl, int A, const void* xfrag, const float* xinit, int64_t n_tiles,
                   int64_t n_points, const void* qhi, const float* qn, const int* qidx,
                   const int* qk, int nq, int kmax, const unsigned* xnmax_bits,
                   const unsigned* bad, int S, int* cand_ids, int* cand_cnt, float* cand_h,
                   void* stream);
// ... slices [s_first, s_first + S_l) of it only (the candidate lists laid out for all S)
int dmlp_screen_x1_part(int KT, int hl, int A, const void* xfrag, const float* xinit,
                        int64_t n_tiles, int64_t n_points, const void* qhi, const float* qn,
                        const int* qidx, const int* qk, int nq, int kmax,
                        const unsigned* xnmax_bits, const unsigned* bad, int S, int s_first,
                        int S_l, int* cand_ids, int* cand_cnt, float* cand_h, void* stream);
// Profiling / tuning switches (process-wide): ablation mode, 4-row group appends on/off,
// sub-buffer depth (8 / 16, 0 = automatic).
void dmlp_set_stream_mode(int mode);
void dmlp_set_stream_groups(int on);
void dmlp_set_stream_sub(int sub);

// ---------------------------------------------------------------- device: exact refine (K2 exact + K3 + K6)
// Exact fp64 distances of the candidates, exact top-k under (dist asc, id desc).
// Writes out_d/out_i[q*kstride + i], i < k_q (rest untouched).  status[q] = 1 if the query
// overflowed and must take the exact fallback path, else 0 (and *ovf_count, if given, grows by
// one per overflowed query: a running total).  Slots [k_q, kstride) get (+inf, -1).  If labels != NULL the vote and
// checksum are fused (out_label[q], out_cs[q]); label_lo/label_hi give the label range.
int dmlp_refine(int cap, const int* cand_ids, const int* cand_cnt, int S, const double* X,
                int A, const double* Qx, const int* qidx, const int* qk, int nq, double* out_d,
                int* out_i, int kstride, const int* labels, int label_lo, int label_hi,
                int* out_label, uint64_t* out_cs, int* status, int* ovf_count, void* stream);
// Same for the single-term screen's group output: members of each group whose single-term score
// (recomputed from xfrag / xinit / qhi, KT in {1,2,4,8}) reaches the (query, slice) threshold cand_h get
// exact distances.  status = 1 also when the survivors exceed 256 (pathological ties).
// qidx may be null: query p is row p (the all-queries pass).
int dmlp_refine_groups(int cap, const int* cand_ids, const int* cand_cnt, const float* cand_h,
                       int S, const double* X, int A, const double* Qx, const void* xfrag,
                       const float* xinit, const void* qhi, int KT, int hl, int64_t n_points,
                       const int* qidx, const int* qk, int nq, double* out_d, int* out_i,
                       int kstride, const int* labels, int label_lo, int label_hi,
                       int* out_label, uint64_t* out_cs, int* status, int* ovf_count, void* stream);
// collect = 1: the lists of dmlp_screen_x1_collect (large k): k <= 256 over <= 512 filtered
// members (fp16 host operands, hl = 1); collect = 0 is dmlp_refine_groups.
int dmlp_refine_groups2(int cap, const int* cand_ids, const int* cand_cnt, const float* cand_h,
                        int S, const double* X, int A, const double* Qx, const void* xfrag,
                        const float* xinit, const void* qhi, int KT, int hl, int64_t n_points,
                        const int* qidx, const int* qk, int nq, double* out_d, int* out_i,
                        int kstride, const int* labels, int label_lo, int label_hi,
                        int* out_label, uint64_t* out_cs, int* status, int* ovf_count,
                        int collect, void* stream);
// dmlp_refine_groups with the image also point-major (xrow, from dmlp_x1_rowmajor; nullptr: none)
// and kmax = the largest k of the list (the two-queries-per-wave kernel serves kmax <= 32 only)
int dmlp_refine_groups_rm(int cap, const int* cand_ids, const int* cand_cnt, const float* cand_h,
                          int S, const double* X, int A, const double* Qx, const void* xfrag,
                          const void* xrow, const float* xinit, const void* qhi, int KT, int hl,
                          int64_t n_points, const int* qidx, const int* qk, int nq, double* out_d,
                          int* out_i, int kstride, const int* labels, int label_lo, int label_hi,
                          int* out_label, uint64_t* out_cs, int* status, int* ovf_count, int kmax,
                          const int* Xi, const int* Qi, void* stream);
// 1 when dmlp_refine_groups_rm serves these lists with the pair refine (which also reads lossless
// int32 rows Xi / Qi instead of X / Qx), 0 when another refine (fp64 rows only)
int dmlp_refine_pair_path(int S, int hl, int KT, int labels, int cap, int kmax);
// the host-rendered fp16 tile image (n_tiles x 64 points x 64 KT bytes) copied point-major
int dmlp_x1_rowmajor(const void* xfrag, int64_t n_tiles, int KT, void* xrow, void* stream);

// Large k on the single-term screen (screen_x1.hip): first-pass thresholds (S1 slices, k' =
// ceil(k / S1)) -> per-query seeds (+inf: a slice overflowed), then the COLLECT pass at those
// fixed thresholds into ccap group ids per (query, slice).
int dmlp_x1_seed(const float* cand_h, const int* cand_cnt, int S1, int nq, float* hseed,
                 void* stream);
int dmlp_screen_x1_collect(int KT, int A, const void* xfrag, const float* xinit, int64_t n_tiles,
                           int64_t n_points, const void* qhi, const float* qn, const int* qidx,
                           const int* qk, int nq, const unsigned* xnmax_bits, const unsigned* bad,
                           const float* hseed, int ccap, int S, int* cand_ids, int* cand_cnt,
                           float* cand_h, void* stream);
// The single-term screen (fp16 host image, S = 1) started while the image is still crossing
// PCIe: rdy[i] != 0 once tiles [i rdy_tiles, (i + 1) rdy_tiles) landed, its value the slice's max
// norm (fp32 bits; a norm of 0 is published as 1); the screen waits per slice (bounded by
// DMLP_EARLY_TIMEOUT_MS of wall clock, default 50: a timed-out wave reports its queries
// overflowed) and grows each column's eps with the slices it has seen.  estats (nullable,
// device, zeroed by the caller): [0] waits that had to spin, [1] eps growths, [2] timeouts,
// summed over the waves.
int dmlp_screen_x1_early(int KT, int A, const void* xfrag, const float* xinit, int64_t n_tiles,
                         int64_t n_points, const void* qhi, const float* qn, const int* qidx,
                         const int* qk, int nq, int kmax, const unsigned* bad, const unsigned* rdy,
                         int rdy_tiles, int rdy_n, int* cand_ids, int* cand_cnt, float* cand_h,
                         unsigned* estats, void* stream);

// ---------------------------------------------------------------- node render plane (plane.cpp)
// P ranks of a node stepping against ONE dataset render it once: slice i of the dataset (image
// tiles + xinit + max norm, and its rows as lossless int32 / fp64) is rendered by rank
// i % renderers into a node-shared page-locked segment and published by a generation flag; every
// rank's dmlp_step (args.plane) copies the slices from there.  The callers separate calls by a
// barrier of all plane ranks.
typedef struct dmlp_plane {
  void* base;       // node-shared segment of >= dmlp_plane_bytes(N, A, with_f64) bytes, set up by
                    // dmlp_plane_init once, page-locked by every rank (dmlp_host_register)
  int64_t bytes;
  int rank;         // this rank among the plane's ranks
  int renderers;    // ranks [0, renderers) render the slices, round-robin (1: rank 0 alone)
  int with_f64;     // fp64 rows region for slices failing the int32 check (else: the node-shared X)
  int pad_;
  int64_t gen;      // this call's generation (> 0, equal on every rank, increasing per call)
  double wait_s;    // bound on a wait for another rank's slice (0: 60 s)
} dmlp_plane;
int dmlp_plane_slices(void);
int64_t dmlp_plane_bytes(int64_t N, int A, int with_f64);
int dmlp_plane_init(void* base, int64_t bytes, int64_t N, int A, int with_f64);
int dmlp_plane_slice(int64_t N, int A, int i, int64_t* t0, int64_t* t1);  // -> slice count
int dmlp_plane_regions(const dmlp_plane* p, int64_t N, int A, void** img, void** xin, void** r32,
                       void** r64);
int dmlp_plane_put_mu(const dmlp_plane* p, int A, const double* mu);
int dmlp_plane_get_mu(const dmlp_plane* p, int A, double* mu);
int dmlp_plane_render(const dmlp_plane* p, const double* X, const double* const* Xr, int64_t N,
                      int A, const double* mu, int what, int i);
int dmlp_plane_wait(const dmlp_plane* p, int what, int i, int* bits, float* nmax);
int dmlp_plane_ready(const dmlp_plane* p, int what, int i);
int dmlp_plane_rows_f64(const dmlp_plane* p, int64_t N, int A, int i, const double* X,
                        double* dst);

// ---------------------------------------------------------------- the native pipeline (pipeline.hip)
// Bump arenas for the pipeline's grow-only buffers, reserved once before any timed call (the
// reference harness times ONE call per process: no hipMalloc may land inside it).  Past the
// reservation allocations fall back to hipMalloc / hipHostMalloc.  Returns 0, | 1 / | 2 when
// the device / host reservation failed.
int dmlp_arena_reserve(int64_t dev_bytes, int64_t host_bytes);
void* dmlp_dev_alloc(int64_t bytes);
void dmlp_dev_free(void* p);
void* dmlp_host_alloc(int64_t bytes);   // page-locked
void dmlp_host_free(void* p);

// Exact local k-NN of device-resident rows X [N][A], Qx [Q][A] with per-query k (host): the
// per-query dispatch (single-term screen k <= 32, 3-term LDS screen k <= 256, exact fp64
// otherwise, per-query escalation of overflows), lists out_d / out_i [Q][kstride] (kstride >= max
// k; (+inf, -1) padding), and with labels (device) the vote + checksum.  exact = 1: the exact
// paths only.  Synchronizes `stream` once (twice when a query escalates).
int dmlp_knn_local(const double* X, int64_t N, int A, const double* Qx, int64_t Q, const int* k,
                   int kstride, double* out_d, int* out_i, const int* labels, int label_lo,
                   int label_hi, int* out_label, uint64_t* out_cs, int exact, void* stream);

// One rank's whole Engine::KNN call from host rows (the call the reference times): host render of
// the screen operands + copies on a side stream (early start when every k is in [1, 32]),
// screens, fp64 rows behind them, exact re-rank, vote, checksum, the report text on the GPU ->
// report_dst (report_mode 1) or kept on the device (report_mode 2: dmlp_step_emit), one host sync.
typedef struct dmlp_step_args {
  const double* X;            // [N][A] row-major, or
  const double* const* Xr;    // [N] row pointers (the drop-in: the harness's own vectors)
  int64_t N;
  int A;
  const int* labels;          // [N]; null: no vote / checksum / report
  int label_lo, label_hi;     // labels in [lo, hi) (hi <= lo: scanned here)
  const double* Qx;           // [Q][A], or
  const double* const* Qr;    // [Q] row pointers
  const int* k;               // [Q]
  int64_t Q;
  int kmin, kmax;             // bounds of k (kmax < kmin: scanned here)
  int64_t qid_base;           // the report's first query id
  int exact;                  // 1: exact fp64 paths only
  int* out_lab;               // device [Q] (null: internal)
  uint64_t* out_cs;           // device [Q] (null: internal)
  double* out_d;              // device [Q][kstride] lists (null: internal)
  int* out_i;
  int kstride;                // >= kmax (0: kmax)
  int report_mode;            // 0 none, 1 -> report_dst, 2 kept on the device
  char* report_dst;           // page-locked, >= dmlp_format_bound(Q) bytes (mode 1)
  int64_t report_cap;
  void* stream;
  const dmlp_plane* plane;    // node render plane (null: this rank renders the whole dataset);
                              // consumers (rank >= renderers) may pass X = Xr = null
  // results
  int64_t report_len;
  int path;                   // 0 host-rendered screen operands, 2 device image (range)
  int early;                  // 1: the screen started before the dataset image landed
  int n_escalated;            // queries redone after a screen overflow
  int early_waits, early_grows, early_timeouts;
  float host_ms;              // host time from entry until every copy / kernel of the call was
                              // issued (the render / pack work and the plane's waits)
  // (input) the dataset's rows already on THIS device as lossless int32 [N][A] (x = m / 1e6: the
  // replica completed over xGMI by an all-gather, parallel/strategies.py "xgmi"): no dataset rows
  // cross PCIe (the host still renders the screen image from X, or the plane does); null: none
  const int* X32d;
} dmlp_step_args;
int dmlp_step(dmlp_step_args* args);
// The last step's device report bytes [0, bytes) -> dst (page-locked / registered), synchronous.
int dmlp_step_emit(char* dst, int64_t bytes, void* stream);
// The device address a report_mode 1 step writes its text to for [p, p + bytes) of page-locked
// host memory, or null when it stages the text on the device and copies it (pageable memory).
void* dmlp_host_device_view(void* p, int64_t bytes, int64_t* info);
// The last dmlp_step's report text as it sits on the device (report_mode 2) and its length.
int dmlp_step_text(const char** dev, int64_t* len);
void dmlp_step_early(int on);          // 1 on, 0 off, < 0: DMLP_FAST_EARLY (default on)
// Right before a timed call after an idle stretch: wake the render pool, touch the staging, keep
// the GPU busy gpu_us microseconds (clocks up).  Synchronous.
int dmlp_step_prewarm(int gpu_us);
void dmlp_step_early_delay(int us);    // host sleep before each image slice (< 0: env)
int dmlp_step_events(int on);          // hipEvent step timeline on / off
int dmlp_step_timeline(double* ms, const char** names, int cap);
// Tuning / A-B switches of the pipeline ("num_cus", "screen", "x1k", "host_ops",
// "device_render"; pipeline.hip
// Tuning): returns the previous value (-1: unknown key).  What the last call did (7 slots): [0]
// exact-path queries, [1] escalated queries, [2] path, [3] early start, [4] exact-path queries on
// the fp64 MFMA screen, [5] of those handed to the fused VALU kernel (overflow), [6] the fp16
// screen operands were rendered on the device (prep.hip k_render).
int dmlp_pipeline_set(const char* key, int value);
void dmlp_pipeline_stats(int64_t* out);

// ---------------------------------------------------------------- device: exact rows (K2, fallback)
// D[i][n] = exact dist(Qx[qidx[i]], X[n]) for i < nq, n < N; ldd = row stride of D (>= N).
int dmlp_exact_rows(const double* X, int64_t N, int A, const double* Qx, const int* qidx, int nq,
                    double* D, int64_t ldd, void* stream);

// Exact top-k of the fallback queries qidx[0..nb): exact rows in descending-id order + stable
// segmented radix sort; k from qk[qidx[i]] (clamped to N); nb*N < 2^31 (callers chunk).
int64_t dmlp_fallback_bytes(int nb, int64_t N);
int dmlp_fallback_topk(const double* X, int64_t N, int A, const double* Qx, const int* qidx,
                       const int* qk, int nb, void* ws, int64_t ws_bytes, double* out_d,
                       int* out_i, int kstride, void* stream);

// Same contract for k <= dmlp_fallback_select_kmax() (2048) by a per-row radix select over the
// exact distance bits + an LDS bitonic sort of the survivors (rows with larger k are skipped;
// callers send those to dmlp_fallback_topk).  Workspace: dmlp_fallback_select_bytes(nb, N).
int dmlp_fallback_select_kmax(void);
// Fused streaming exact top-k (exact.hip), k <= dmlp_exact_topk_kmax(): no workspace, no
// distance rows; kmax bounds the k of these queries.
int dmlp_exact_topk_kmax(void);
int dmlp_exact_topk_kmax_for(int64_t N);  // dispatch policy: fused vs rows + select
int dmlp_exact_topk(const double* X, int64_t N, int A, const double* Qx, const int* qidx,
                    const int* qk, int nb, int kmax, double* out_d, int* out_i, int kstride,
                    void* stream);
int64_t dmlp_fallback_select_bytes(int nb, int64_t N);
int dmlp_fallback_select(const double* X, int64_t N, int A, const double* Qx, const int* qidx,
                         const int* qk, int nb, void* ws, int64_t ws_bytes, double* out_d,
                         int* out_i, int kstride, void* stream);

// ---------------------------------------------------------------- device: top-k merge (K4)
// L sorted lists per query (list l of query q at in_*[l*list_stride + q*kin + j]), padded with
// (+inf, -1).  Writes the merged top-k_q of every query q < nq to out_*[q*kout + i].
int dmlp_merge(const double* in_d, const int* in_i, int L, int64_t list_stride, int kin,
               const int* qk, int nq, double* out_d, int* out_i, int kout, void* stream);

// ---------------------------------------------------------------- device: vote + checksum (K5, K7)
// Rows qidx[i] (or i if qidx == NULL), i < nq.
int dmlp_finalize(const double* d, const int* ids, int kstride, const int* qk, const int* qidx,
                  int nq, const int* labels, int label_lo, int label_hi, int* out_label,
                  uint64_t* out_cs, void* stream);

int dmlp_fill_f64(double* p, int64_t n, double v, void* stream);
int dmlp_offset_ids(int* ids, int64_t n, int off, void* stream);

// ---------------------------------------------------------------- device: report formatting (K7)
// "Query <qid> checksum: <cs>\n" for q < nq into out (needs dmlp_format_bound bytes).
// line_off[dmlp_format_scratch(nq)] is int64 scratch: line_off[0..nq] receives the line offsets
// (line_off[nq] = total bytes), the tail holds the per-block sums of the scan.
int64_t dmlp_format_bound(int nq);
int64_t dmlp_format_scratch(int nq);
int dmlp_format_report(const uint64_t* cs, int nq, int qid_base, int64_t* line_off, char* out,
                       void* stream);
// ... with the lines starting at byte *base of out (base: device int64, null = 0); line_off then
// holds absolute offsets (line_off[nq] = the end of this run's text)
int dmlp_format_report_at(const uint64_t* cs, int nq, int qid_base, int64_t* line_off, char* out,
                          const int64_t* base, void* stream);

// ---------------------------------------------------------------- host (CPU) implementations
int dmlp_cpu_knn(const double* X, int64_t N, int A, const double* Qx, int64_t Q, const int* qk,
                 int kstride, double* out_d, int* out_i, int nthreads);
int dmlp_cpu_finalize(const double* d, const int* ids, int kstride, const int* qk, int64_t Q,
                      const int* labels, int* out_label, uint64_t* out_cs);
int dmlp_cpu_merge(const double* in_d, const int* in_i, int L, int64_t list_stride, int kin,
                   const int* qk, int64_t Q, double* out_d, int* out_i, int kout);
int dmlp_kdtree_knn(const double* X, int64_t N, int A, const double* Qx, int64_t Q,
                    const int* qk, int kstride, double* out_d, int* out_i);
// Text report, host side.  Returns bytes written (buffer must hold 48*Q bytes).
void dmlp_cpu_i32_range(const int* a, int64_t n, int* lo, int* hi);
void dmlp_host_i32_range(const int* a, int64_t n, int* lo, int* hi);  // on the render pool
int64_t dmlp_atomic_fetch_add_i64(int64_t* p, int64_t v);
void dmlp_atomic_store_i64(int64_t* p, int64_t v);
int64_t dmlp_cpu_format_report(const uint64_t* cs, int64_t Q, int64_t qid_base, char* out);
int64_t dmlp_cpu_format_debug(const double* d, const int* ids, int kstride, const int* qk,
                              const int* labels_pred, int64_t Q, char* out, int64_t cap);

// ---------------------------------------------------------------- host: input parsing (common.cpp:12-44)
// Parses the header.  Returns 0 on success.
int dmlp_parse_header(const char* buf, int64_t len, int64_t* N, int64_t* Q, int* A,
                      int64_t* body_off);
// Parses N data lines and Q query lines starting at body_off (multi-threaded).
// Returns 0, or -(line_no+1) of the first malformed line.
int64_t dmlp_parse_body(const char* buf, int64_t len, int64_t body_off, int64_t N, int64_t Q,
                        int A, int* labels, double* X, int* qk, double* Qx, int nthreads);

// Page-lock / unlock an existing host range (node-shared input segments).  0 or a hipError_t.
int dmlp_host_register(void* p, int64_t bytes);
int dmlp_host_unregister(void* p);

// The reference's input file (generate_input.py's format, "%.6f" attributes) from arrays,
// formatted on the render pool.  0 or -1.
int dmlp_cpu_write_input(const char* path, const int* labels, const double* X, int64_t N,
                         const int* k, const double* Qx, int64_t Q, int A);

const char* dmlp_version(void);
int dmlp_device_count(void);

#ifdef __cplusplus
}
#endif
