// refine.hip — exact re-ranking, top-k merge, vote/checksum and report formatting.
//
//  * k_refine   : exact fp64 distances (reference order, no FMA: engine.cpp:12-18) of the
//                 screen's survivors and an exact top-k under (dist asc, id desc)
//                 (SURVEY.md §2.5 K2/K3/K6).  One wave per query; a P-slot running top-k in
//                 LDS absorbs 64 candidates per step and is re-sorted (register bitonic) only
//                 when full.  Vote + FNV checksum are fused when labels are given (K5/K7).
//  * k_merge    : K-way merge of sorted per-shard top-k lists — the device analog of bench_2's
//                 user MPI_Op (@0xbc70) and bench_1's root sort (@0xdae6); RCCL has no user
//                 reductions, so strategies call this between send/recv rounds (K4).
//                 L <= 8 lists: k_merge_seq (one lane per query, heads in registers);
//                 more: k_merge_path (LDS merge path) or the rank kernel.
//  * k_finalize : vote (max count, tie -> larger label; engine.cpp:319-332) + FNV-1a checksum
//                 (common.cpp:59-70) of sorted lists.
//  * k_exact_rows: full exact distance rows (fallback for k > screen kmax, overflowing queries,
//                 or data outside the screen's range).
//  * k_format_* : "Query <id> checksum: <u64>\n" rendered on the GPU (common.cpp:70).
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

#include <algorithm>

namespace {

constexpr int kHistCap = 512;  // per-wave label histogram (labels in [lo, lo+512))

// the same over a lossless int32 row, each value divided back exactly as k_rows_from_i32 does
__device__ __forceinline__ double exact_dist_row_i32(const double* __restrict__ q,
                                                     const int* __restrict__ x, int A) {
  double s = 0.0;
  for (int a = 0; a < A; ++a) {
    const double d = __dsub_rn(q[a], (double)x[a] / 1.0e6);
    s = __dadd_rn(s, __dmul_rn(d, d));
  }
  return s;
}

__device__ __forceinline__ double exact_dist_row(const double* __restrict__ q,
                                                 const double* __restrict__ x, int A) {
  double s = 0.0;
  if ((A & 1) == 0) {
    const double2* x2 = (const double2*)x;
    for (int a = 0; a < (A >> 1); ++a) {
      const double2 v = x2[a];
      const double d0 = __dsub_rn(q[2 * a], v.x);
      s = __dadd_rn(s, __dmul_rn(d0, d0));
      const double d1 = __dsub_rn(q[2 * a + 1], v.y);
      s = __dadd_rn(s, __dmul_rn(d1, d1));
    }
  } else {
    for (int a = 0; a < A; ++a) {
      const double d = __dsub_rn(q[a], x[a]);
      s = __dadd_rn(s, __dmul_rn(d, d));
    }
  }
  return s;
}

// Running top-k of one wave, P = E*64 slots in LDS: [0,k) current best (sorted), new
// candidates appended at k+fill; re-sorted when fewer than 64 free slots remain.
template <int E>
struct RunTopK {
  static constexpr int P = E * 64;
  double* d;
  int* id;
  int k;
  int fill;
  __device__ void init(double* d_, int* id_, int k_) {
    d = d_; id = id_; k = k_; fill = 0;
    for (int i = dmlp::lane_id(); i < P; i += 64) { d[i] = INFINITY; id[i] = -1; }
    dmlp::wave_sync();
  }
  __device__ void flush() {
    if (fill == 0) return;
    double rd[E]; int ri[E];
    const int lane = dmlp::lane_id();
    dmlp::wave_sync();
#pragma unroll
    for (int r = 0; r < E; ++r) { rd[r] = d[r * 64 + lane]; ri[r] = id[r * 64 + lane]; }
    dmlp::wave_sort_keys<E>(rd, ri);
    dmlp::wave_sync();
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int i = r * 64 + lane;
      d[i] = i < k ? rd[r] : INFINITY;
      id[i] = i < k ? ri[r] : -1;
    }
    dmlp::wave_sync();
    fill = 0;
  }
  __device__ void push(bool valid, double dv, int iv) {
    const unsigned long long m = __ballot(valid);
    if (valid) {
      const int pos = k + fill + __popcll(m & dmlp::lanemask_lt());
      d[pos] = dv;
      id[pos] = iv;
    }
    fill += __popcll(m);
    if (k + fill + 64 > P) flush();
  }
};

__device__ __forceinline__ void finalize_wave(const int* ids, int k, const int* __restrict__ labels,
                                              int label_lo, int label_hi, int* hist,
                                              int* out_label, uint64_t* out_cs,
                                              int hist_cap = kHistCap) {
  const int lane = dmlp::lane_id();
  // labels of ids < 0 (padding) are never read
  const int label = k > 0 ? dmlp::wave_vote(ids, k, labels, label_lo, label_hi, hist, hist_cap) : -1;
  if (lane == 0) {
    *out_label = label;
    *out_cs = dmlp::fnv_checksum(label, ids, k);
  }
}

// Group-mode inputs (single-term screen, screen_x1.hip): candidates are 4-row group entries
// (ordered 16-bit group-max key << 16 | slice-relative group index) and cand_h holds each
// slice's final threshold and the query's screen error bound eps.  The k-th largest key over all slices gives h = a_k' - 2 eps (a lower
// bound on a_k - eps, exactly the screen's own rule, but global); a member survives iff its
// single-term score  s = -|x'|^2/2 + <hi(q'), hi(x')>  (recomputed from the screen's image: bf16
// for hl = 2, fp16 for hl = 1;
// any summation order obeys the same error bound) is >= h.  Only survivors get exact distances.
struct GroupIn {
  const float* cand_h;    // [nq * S][2]: slice threshold, query eps
  const u32x4* xfrag;     // tile image (hi first; hl = 2: prep.hip's hi/lo, 1: hi only)
  const float* xinit;     // -|x'|^2/2 per point
  const bf16x8* qhi;      // [Q][KT*4] query hi fragments
  int KT;
  int hl;
  int n_points;
  int tiles_per_slice;    // the screen's slicing: group base = (s * tps * 64) + 4 * index
  int collect;            // lists of the COLLECT pass (large k): the threshold is always taken
                          // over the lists (cand_h holds the fixed seed, not a final threshold)
  int rescore = 1;        // 0 (screen_f64.hip's fp64 keys): every member of a group at or above
                          // the threshold goes to the exact re-rank (no image to rescore from)
  int grows = 4;          // rows per group entry: 4 (consecutive) or 8 (the SUB = 16 screen's pair
                          // epilogue: rows 4 kg + i of steps 2p and 2p + 1, entry = 4 p + kg)
  const int* xi32 = nullptr;  // the dataset's lossless int32 rows (X unused), or null
};

// row of member i (< grows) of the group with slice-relative entry index gi
__device__ __forceinline__ int group_row(unsigned gi, int i, int grows) {
  return grows == 8 ? (int)(gi >> 2) * 32 + (int)(gi & 3) * 4 + ((i & 4) << 2) + (i & 3)
                    : (int)gi * 4 + i;
}

// GROUPS = KT of the single-term screen (1, 2, 4 or 8) for group-mode input, 0 otherwise.  The group
// variant sizes its LDS for k <= 32 (the screen's limit) and labels in [lo, lo + 256) (wider
// label ranges take wave_vote's counting fallback), so more waves stay resident to hide the
// gathers that dominate this kernel.
// E = 8 with GROUPS: the large-k group variant (k <= 256 over <= 512 filtered members): its
// top-k is one wave-wide bitonic sort of the members' exact keys, and labels are gathered at the
// vote (no carry scratch).
template <int E, int GROUPS, bool F16 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((GROUPS && E >= 8) ? 2 : GROUPS == 1 ? 8 : GROUPS ? 4 : 1))) void k_refine(
    const int* __restrict__ cand_ids, const int* __restrict__ cand_cnt, int S, int cap,
    const double* __restrict__ X, int A, const double* __restrict__ Qx,
    const int* __restrict__ qidx, const int* __restrict__ qk, int nq, double* __restrict__ out_d,
    int* __restrict__ out_i, int kstride, const int* __restrict__ labels, int label_lo,
    int label_hi, int* __restrict__ out_label, uint64_t* __restrict__ out_cs,
    int* __restrict__ status, int* __restrict__ ovf_count, const GroupIn gin) {
  constexpr int P = E * 64;
  constexpr int SMAX = 256;
  constexpr bool GBIG = GROUPS && E >= 8;
  constexpr int KMAX = GBIG ? 256 : GROUPS ? 64 : 128;
  constexpr int HCAP = GROUPS ? 256 : kHistCap;  // >= 256: the key histogram of the global threshold
  __shared__ double s_d[4][P];
  __shared__ int s_i[4][P];
  __shared__ double s_rd[4][KMAX];
  __shared__ int s_ri[4][KMAX];
  __shared__ int s_pre[4][SMAX + 1];
  __shared__ __attribute__((aligned(16))) int s_hist[4][HCAP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int p = blockIdx.x * 4 + wave;
  if (p >= nq) return;
  // qidx == nullptr: every query in order (no dependent index load at the head of the chain)
  const int q = qidx ? __builtin_amdgcn_readfirstlane(qidx[p]) : p;
  const int k = __builtin_amdgcn_readfirstlane(qk[q]);
  const int* cnt = cand_cnt + (int64_t)p * S;
  // group mode: everything that depends only on (p, q) is requested here, in one batch, instead
  // of one dependent latency after another (this kernel is bound by its chain of gathers)
  constexpr int KTG = GROUPS ? GROUPS : 1;
  // A > 64 (KT = 4, 8): hi(q') is read from LDS at each use (staged below) — 64 / 128 registers
  // held through the member loop would spill
  constexpr bool QLDS = GROUPS >= 4;
  u32x4 qraw[QLDS ? 1 : KTG * 4];
  float g_eps = 0.0f, g_h1 = 0.0f;
  unsigned ebuf = 0;  // S == 1: entry `lane` of the query's single slice
  if (GROUPS) {
    if (KTG == 1 && gin.rescore) {  // (KT = 2: 32 registers held this long would spill; loaded at first use)
#pragma unroll
      for (int f = 0; f < KTG * 4; ++f)
        qraw[f] = __builtin_bit_cast(u32x4, gin.qhi[(int64_t)q * KTG * 4 + f]);
    }
    g_eps = gin.cand_h[2 * (int64_t)p * S + 1];
    g_h1 = gin.cand_h[2 * (int64_t)p * S];  // slice 0's (COLLECT: every slice holds the seed)
    if (S == 1 && lane < cap) ebuf = (unsigned)cand_ids[(int64_t)p * cap + lane];
  }
  // prefix of candidate counts over slices (S <= SMAX); group mode: the largest eps over the
  // slices — a screen launched per data chunk (pipeline.hip's large-N pipeline) bounds each
  // slice's error with the image's max norm seen so far, and the global threshold must hold for
  // every slice's members (a_k' - 2 max eps <= a_k - eps of any member)
  int* pre = s_pre[wave];
  bool ovf = false;
  if (lane == 0) {
    int acc = 0;
    pre[0] = 0;
    for (int s = 0; s < S; ++s) {
      const int n = cnt[s];
      if (n < 0) ovf = true;
      acc += n < 0 ? 0 : n;
      pre[s + 1] = acc;
      if (GROUPS && s > 0) g_eps = fmaxf(g_eps, gin.cand_h[2 * ((int64_t)p * S + s) + 1]);
    }
  }
  ovf = __shfl(ovf ? 1 : 0, 0) != 0;
  if (GROUPS) g_eps = __shfl(g_eps, 0);
  // the (+inf, -1) padding of slots [k, kstride) is written here, so callers need no fill pass
  // (slots [0, k) of a query handed back below are written by its escalation / exact path)
  for (int i = k + lane; i < kstride; i += 64) {
    out_d[(int64_t)q * kstride + i] = INFINITY;
    out_i[(int64_t)q * kstride + i] = -1;
  }
  if (ovf) {
    if (lane == 0) {
      status[q] = 1;
      if (ovf_count) atomicAdd(ovf_count, 1);  // running total: the host reads 4 bytes
    }
    return;
  }
  if (lane == 0) status[q] = 0;
  dmlp::wave_sync();
  int M = pre[S];
  const double* qv = Qx + (int64_t)q * A;
  auto slice_of = [&](int j) {
    // slice containing flat index j: largest s with pre[s] <= j
    int lo = 0, hi = S;  // pre[lo] <= j < pre[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (pre[mid] <= j) lo = mid; else hi = mid;
    }
    return lo;
  };
  auto cand = [&](int j, double& dv, int& id) {
    if (GROUPS) {
      id = s_i[wave][j];  // filtered members, staged below
    } else {
      const int lo = slice_of(j);
      id = cand_ids[((int64_t)p * S + lo) * cap + (j - pre[lo])];
    }
    dv = gin.xi32 ? exact_dist_row_i32(qv, gin.xi32 + (int64_t)id * A, A)
                  : exact_dist_row(qv, X + (int64_t)id * A, A);
  };
  if (GROUPS) {
    // ---- global threshold: k-th largest group key over all slices (two 8-bit histogram passes)
    auto entry = [&](int j) {
      const int lo = slice_of(j);
      return (unsigned)cand_ids[((int64_t)p * S + lo) * cap + (j - pre[lo])];
    };
    int* hist = s_hist[wave];
    const float eps = g_eps;
    // one slice: its final threshold is already global; COLLECT lists: the fixed seed (a valid
    // bound every slice shares), raised below to the k-th largest key over the lists
    float hq = S == 1 || gin.collect ? g_h1 : -INFINITY;
    if ((S > 1 || gin.collect) && M >= k && k >= 1) {
      int above = 0;
      int b1 = -1, b2 = -1;
#pragma unroll 1
      for (int pass = 0; pass < 2; ++pass) {
        for (int i = lane; i < 256; i += 64) hist[i] = 0;
        dmlp::wave_sync();
        for (int j = lane; j < M; j += 64) {
          const unsigned e = entry(j);
          if (pass == 0) atomicAdd(&hist[e >> 24], 1);
          else if ((int)(e >> 24) == b1) atomicAdd(&hist[(e >> 16) & 255], 1);
        }
        dmlp::wave_sync();
        const int b = dmlp::wave_kth_bin(hist, k - above, above);
        dmlp::wave_sync();
        if (pass == 0) b1 = b; else b2 = b;
      }
      const unsigned T = ((unsigned)b1 << 24) | ((unsigned)b2 << 16);
      const unsigned tb = T ^ ((T >> 31) ? 0x80000000u : 0xffffffffu);  // ordered -> fp32 bits
      hq = fmaxf(hq, __uint_as_float(tb) - 2.0f * eps);
    }
    const unsigned tq = __float_as_uint(hq);
    const unsigned kh = (tq ^ ((unsigned)((int)tq >> 31) | 0x80000000u)) & 0xffff0000u;
    // ---- expand surviving groups; keep members whose single-term score reaches hq
    constexpr int KT = GROUPS ? GROUPS : 1;  // (dead code for GROUPS == 0)
    // hi(q') stays packed (two bf16 per dword, 16 VGPRs per KT): unpacked at each use — a
    // 32-float copy would push this 64-register kernel into scratch spills
    u32x4* const qs = (u32x4*)s_hist[wave];  // (the histogram is dead once hq is known)
    if constexpr (QLDS) {
      static_assert(KT * 4 * 16 <= HCAP * 4, "query fragments must fit the histogram scratch");
      for (int f = lane; f < KT * 4 && gin.rescore; f += 64)
        qs[f] = __builtin_bit_cast(u32x4, gin.qhi[(int64_t)q * KT * 4 + f]);
      dmlp::wave_sync();
    } else if (KT != 1 && gin.rescore) {
#pragma unroll
      for (int f = 0; f < KT * 4; ++f)
        qraw[f] = __builtin_bit_cast(u32x4, gin.qhi[(int64_t)q * KT * 4 + f]);
    }
    // one member per lane (4 lanes per group: their fragments are adjacent 16-byte chunks).
    // Entries are fetched 64 groups at a time, one per lane, and dealt to the member lanes by
    // a shuffle: each 64-member step then waits on one gather (the fragments), not two.
    int nm = 0;
    const int GR = gin.grows, GS = GR == 8 ? 3 : 2;  // members per group entry, log2
    for (int j0 = 0; j0 < GR * M; j0 += 64) {
      const int jm = j0 + lane;
      const int g = jm >> GS;
      // S == 1: block 0 was fetched up front
      if ((j0 & (64 * GR - 1)) == 0 && (S > 1 || j0 > 0)) {
        const int gg = (j0 >> GS) + lane;
        ebuf = 0;
        if (gg < M) {
          const int lo = slice_of(gg);
          ebuf = (unsigned)cand_ids[((int64_t)p * S + lo) * cap + (gg - pre[lo])];
        }
      }
      const unsigned e = (unsigned)__shfl((int)ebuf, g & 63);
      int id = 0;
      bool keep = false;
      if (g < M) {
        const int lo = slice_of(g);
        id = lo * gin.tiles_per_slice * 64 + group_row(e & 0xffffu, jm & (GR - 1), GR);
        if (e >= kh && id < gin.n_points && !gin.rescore) {
          keep = true;
        } else if (e >= kh && id < gin.n_points) {
          const int64_t t = id >> 6;
          const int pl = id & 63;
          const u32x4* fr = gin.xfrag + t * (int64_t)(4 * KT * gin.hl * 64) + (pl & 15);
          float sc = gin.xinit[id];
          // F16: the host's fp16 image + fp16 query fragments (hl = 1); else bf16 (a template
          // parameter: both decodes in one body pushed this 64-VGPR kernel into scratch spills)
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) {
            const u32x4* fk = fr + (int64_t)(((pl >> 4) * KT + kt) * gin.hl) * 64;
#pragma unroll
            for (int kq = 0; kq < 4; ++kq) {
              const u32x4 w = fk[16 * kq];
              const u32x4 qv = QLDS ? qs[kt * 4 + kq] : qraw[QLDS ? 0 : kt * 4 + kq];
#pragma unroll
              for (int q2 = 0; q2 < 4; ++q2) {
                const unsigned qw = qv[q2];
                if constexpr (F16) {  // products exact in fp32 either way: any order obeys the bound
                  sc += (float)__builtin_bit_cast(_Float16, (unsigned short)(qw & 0xffffu)) *
                        (float)__builtin_bit_cast(_Float16, (unsigned short)(w[q2] & 0xffffu));
                  sc += (float)__builtin_bit_cast(_Float16, (unsigned short)(qw >> 16)) *
                        (float)__builtin_bit_cast(_Float16, (unsigned short)(w[q2] >> 16));
                } else {
                  sc += __uint_as_float(qw << 16) * __uint_as_float(w[q2] << 16);
                  sc += __uint_as_float(qw & 0xffff0000u) * __uint_as_float(w[q2] & 0xffff0000u);
                }
              }
            }
          }
          keep = sc >= hq;
        }
      }
      const unsigned long long km = __ballot(keep);
      const int pos = nm + __popcll(km & dmlp::lanemask_lt());
      if (keep && pos < P) s_i[wave][pos] = id;
      nm += __popcll(km);
    }
    if (nm > P) {
      // pathological ties: hand the query back (x1 overflow -> 3-term screen escalation)
      if (lane == 0) {
        status[q] = 1;
        if (ovf_count) atomicAdd(ovf_count, 1);
      }
      return;
    }
    M = nm;
    dmlp::wave_sync();
  }
  const double* res_d;
  const int* res_i;
  // group mode: each candidate's label is gathered beside its row and travels with it (in the
  // slice-prefix scratch, dead after the member filter), so the vote reads LDS, not a final
  // dependent gather.  cl: candidates' labels [P], rl: the top-k's labels [KMAX].
  const bool carry = GROUPS && !GBIG && labels != nullptr;
  int* const cl = s_pre[wave];
  int* const rl = s_pre[wave] + P;
  static_assert(!GROUPS || GBIG || P + KMAX <= SMAX + 1, "label scratch must fit the prefix array");
  bool carried = false;
  if constexpr (GBIG) {
    // M <= P filtered members (checked above): exact keys, one bitonic sort, the first k
    double rd[E];
    int ri[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int j = r * 64 + lane;
      rd[r] = INFINITY;
      ri[r] = -1;
      if (j < M) cand(j, rd[r], ri[r]);
    }
    dmlp::wave_sync();  // every member id read before the sorted keys overwrite the arrays
    dmlp::wave_sort_keys<E>(rd, ri);
#pragma unroll
    for (int r = 0; r < E; ++r) {
      s_d[wave][r * 64 + lane] = rd[r];
      s_i[wave][r * 64 + lane] = ri[r];
    }
    dmlp::wave_sync();
    res_d = s_d[wave];
    res_i = s_i[wave];
  } else if (M <= P && k <= KMAX) {
    // rank select: keys are unique (distinct ids), so rank(i) = #{j : key_j < key_i} places
    // every member of the top-k directly at its sorted position.
    double* cd = s_d[wave];
    int* ci = s_i[wave];
    for (int j = lane; j < M; j += 64) {
      double dv; int id;
      cand(j, dv, id);
      if (carry) cl[j] = labels[id];
      cd[j] = dv;
      if (!GROUPS) ci[j] = id;
    }
    carried = carry;
    for (int i = lane; i < k; i += 64) { s_rd[wave][i] = INFINITY; s_ri[wave][i] = -1; }
    dmlp::wave_sync();
    int Ms = M;
    if (M > 64 && k <= 64) {
      // O(M^2) ranking is the cost when the screen hands over a few hundred ids (4-row group
      // mode): the k-th smallest key of ANY subset bounds the k-th smallest of all from above,
      // so rank the first 64 candidates, keep only keys <= that bound (always >= k of them,
      // every true top-k member among them), and rank the survivors.
      const double di = cd[lane];
      const int ii = ci[lane];
      int rank = 0;
#pragma unroll 32
      for (int j = 0; j < 64; ++j) rank += dmlp::key_less(cd[j], ci[j], di, ii) ? 1 : 0;
      const unsigned long long hit = __ballot(rank == k - 1);
      const int src = __ffsll((long long)hit) - 1;
      const double td = __shfl(di, src);
      const int ti = __shfl(ii, src);
      dmlp::wave_sync();
      int kept = 0;
      for (int j0 = 0; j0 < M; j0 += 64) {
        const int j = j0 + lane;
        double dj = INFINITY;
        int ij = -1, lj = 0;
        bool keep = false;
        if (j < M) {
          dj = cd[j];
          ij = ci[j];
          if (carry) lj = cl[j];
          keep = !dmlp::key_less(td, ti, dj, ij);  // key_j <= bound
        }
        const unsigned long long km = __ballot(keep);
        dmlp::wave_sync();  // slots < j0 + 64 already read by every lane
        if (keep) {
          const int pos = kept + __popcll(km & dmlp::lanemask_lt());
          cd[pos] = dj;
          ci[pos] = ij;
          if (carry) cl[pos] = lj;
        }
        kept += __popcll(km);
      }
      dmlp::wave_sync();
      Ms = kept;
    }
    for (int i = lane; i < Ms; i += 64) {
      const double di = cd[i];
      const int ii = ci[i];
      int rank = 0;
#pragma unroll 32
      for (int j = 0; j < Ms; ++j) rank += dmlp::key_less(cd[j], ci[j], di, ii) ? 1 : 0;
      if (rank < k) {
        s_rd[wave][rank] = di;
        s_ri[wave][rank] = ii;
        if (carry) rl[rank] = cl[i];
      }
    }
    dmlp::wave_sync();
    res_d = s_rd[wave];
    res_i = s_ri[wave];
  } else {
    RunTopK<E> tk;
    tk.init(s_d[wave], s_i[wave], k);
    for (int j0 = 0; j0 < M; j0 += 64) {
      const int j = j0 + lane;
      const bool valid = j < M;
      int id = 0;
      double dv = INFINITY;
      if (valid) cand(j, dv, id);
      tk.push(valid, dv, id);
    }
    tk.flush();
    res_d = tk.d;
    res_i = tk.id;
  }
  for (int i = lane; i < k; i += 64) {
    out_d[(int64_t)q * kstride + i] = res_d[i];
    out_i[(int64_t)q * kstride + i] = res_i[i];
  }
  if (labels) {
    dmlp::wave_sync();
    if (carried) {
      const int label = k > 0 ? dmlp::wave_vote_by(res_i, k, [&](int i, int) { return rl[i]; },
                                                   label_lo, label_hi, s_hist[wave], HCAP)
                              : -1;
      if (lane == 0) {
        out_label[q] = label;
        out_cs[q] = dmlp::fnv_checksum(label, res_i, k);
      }
    } else {
      finalize_wave(res_i, k, labels, label_lo, label_hi, s_hist[wave], out_label + q,
                    out_cs + q, HCAP);
    }
  }
}

// K-way merge of L sorted top-k lists per query (K4: bench_2's custom MPI_Op / bench_1's root
// merge), one wave per query, no sequential head scan: every element's output position is its
// rank in the union, i.e. its index in its own list plus, for every other list, the number of
// entries ordered before it (a binary search over that list's real prefix; ties between lists
// go to the lower list index).  The ranks of the real elements are therefore exactly
// 0 .. total-1; each element with rank < k is stored once, and slots [total, k) get the
// (+inf, -1) padding.  Padding entries (id < 0) form a suffix of each list.
__global__ __launch_bounds__(256) void k_merge(const double* __restrict__ in_d,
                                               const int* __restrict__ in_i, int L,
                                               int64_t list_stride, int kin,
                                               const int* __restrict__ qk, int nq,
                                               double* __restrict__ out_d, int* __restrict__ out_i,
                                               int kout) {
  __shared__ int s_cnt[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x * 4 + wave;
  if (q >= nq) return;
  int k = qk[q];
  k = k < kout ? k : kout;
  const int lim = k < kin ? k : kin;
  const int64_t qo = (int64_t)q * kin;
  int* cnt = s_cnt[wave];
  // real prefix length of each list (first padding entry, by binary search)
  for (int l = lane; l < L; l += 64) {
    const int* ids = in_i + l * list_stride + qo;
    int lo = 0, n = lim;
    while (n > 0) {
      const int h = n >> 1;
      if (ids[lo + h] >= 0) { lo += h + 1; n -= h + 1; } else { n = h; }
    }
    cnt[l] = lo;
  }
  dmlp::wave_sync();
  int total = 0;
  for (int l = 0; l < L; ++l) total += cnt[l];
  for (int t = lane; t < L * lim; t += 64) {
    const int l = t / lim, p = t - l * lim;
    if (p >= cnt[l]) continue;
    const int64_t off = l * list_stride + qo + p;
    const double d = in_d[off];
    const int id = in_i[off];
    int rank = p;
    for (int m = 0; m < L && rank < k; ++m) {
      if (m == l) continue;
      const double* md = in_d + m * list_stride + qo;
      const int* mi = in_i + m * list_stride + qo;
      // equal keys (only when the caller's lists overlap) order by list index, as a sequential
      // merge that scans the lists in order would: count entries <= the key in earlier lists
      const bool before = m < l;
      int lo = 0, n = cnt[m];
      while (n > 0) {
        const int h = n >> 1;
        const bool lt = before ? !dmlp::key_less(d, id, md[lo + h], mi[lo + h])
                               : dmlp::key_less(md[lo + h], mi[lo + h], d, id);
        if (lt) { lo += h + 1; n -= h + 1; } else { n = h; }
      }
      rank += lo;
    }
    if (rank < k) {
      out_d[(int64_t)q * kout + rank] = d;
      out_i[(int64_t)q * kout + rank] = id;
    }
  }
  for (int o = total + lane; o < k; o += 64) {
    out_d[(int64_t)q * kout + o] = INFINITY;
    out_i[(int64_t)q * kout + o] = -1;
  }
}

// Merge-path form of the same K4 merge for lists that fit in LDS (2 x L x kout entries):
// one wave per query stages the L real prefixes in LDS, then merges adjacent pairs level by
// level (log2 L levels, ties to the lower list index, i.e. the earlier pair member — the same
// order as the rank kernel).  Every output element of a pair merge finds its co-rank (how many
// of its predecessors come from the first list) by one binary search, so a lane does
// ceil(pairs x k / 64) searches of log2 k probes per level, all in LDS.
__global__ __launch_bounds__(256) void k_merge_path(const double* __restrict__ in_d,
                                                   const int* __restrict__ in_i, int L,
                                                   int64_t list_stride, int kin,
                                                   const int* __restrict__ qk, int nq,
                                                   double* __restrict__ out_d,
                                                   int* __restrict__ out_i, int kout, int lcap) {
  extern __shared__ __attribute__((aligned(16))) char smem_all[];
  __shared__ int s_cnt_all[4][2][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x * (blockDim.x >> 6) + wave;  // one query per wave
  if (q >= nq) return;
  char* const smem = smem_all + (size_t)wave * 2 * L * lcap * (sizeof(double) + sizeof(int));
  int (*s_cnt)[64] = s_cnt_all[wave];
  int k = qk[q];
  k = k < kout ? k : kout;
  const int lim = k < kin ? k : kin;
  double* bd[2] = {(double*)smem, (double*)smem + (size_t)L * lcap};
  int* bi[2] = {(int*)((double*)smem + 2 * (size_t)L * lcap),
                (int*)((double*)smem + 2 * (size_t)L * lcap) + (size_t)L * lcap};
  const int64_t qo = (int64_t)q * kin;
  // t / d for the small flat indices below by a float reciprocal (exact: t < 2^16, +0.5 margin)
  auto divq = [](int t, float inv) { return (int)(((float)t + 0.5f) * inv); };
  // stage the L prefixes (all loads of a lane issued back to back), then each list's real
  // prefix length by a binary search for its first padding id
  const float inv_lim = 1.0f / (float)(lim > 0 ? lim : 1);
  for (int t0 = 0; t0 < L * lim; t0 += 256) {  // 4 loads in flight per lane, then the stores
    double dv[4];
    int iv[4], dst[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 64 * u + lane;
      dst[u] = -1;
      if (t < L * lim) {
        const int l = divq(t, inv_lim), p = t - l * lim;
        const int64_t off = l * list_stride + qo + p;
        dv[u] = in_d[off];
        iv[u] = in_i[off];
        dst[u] = l * lcap + p;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (dst[u] >= 0) { bd[0][dst[u]] = dv[u]; bi[0][dst[u]] = iv[u]; }
  }
  dmlp::wave_sync();
  for (int l = lane; l < L; l += 64) {
    const int* ids = bi[0] + l * lcap;
    int lo = 0, n = lim;
    while (n > 0) {
      const int h = n >> 1;
      if (ids[lo + h] >= 0) { lo += h + 1; n -= h + 1; } else { n = h; }
    }
    s_cnt[0][l] = lo;
  }
  dmlp::wave_sync();
  const float inv_k = 1.0f / (float)(k > 0 ? k : 1);
  int cur = 0, Lc = L;
  while (Lc > 1) {
    const int Ln = (Lc + 1) >> 1;
    const double* sd = bd[cur];
    const int* si = bi[cur];
    double* dd = bd[cur ^ 1];
    int* di = bi[cur ^ 1];
    // lane-contiguous output ranges over the flattened (pair, position) space: one co-rank
    // search per pair segment, then a sequential merge of the segment from register heads
    const int tot = Ln * k;
    const int chunk = (tot + 63) >> 6;
    int t = lane * chunk;
    const int tend = t + chunk < tot ? t + chunk : tot;
    while (t < tend) {
      const int pr = divq(t, inv_k), o0 = t - pr * k;
      const int oend = o0 + (tend - t) < k ? o0 + (tend - t) : k;
      t += oend - o0;
      const int la = 2 * pr, lb = la + 1;
      const int ca = s_cnt[cur][la];
      const double* ad = sd + la * lcap;
      const int* ai = si + la * lcap;
      double* od = dd + pr * lcap;
      int* oi = di + pr * lcap;
      if (lb >= Lc) {
        for (int o = o0; o < oend && o < ca; ++o) { od[o] = ad[o]; oi[o] = ai[o]; }
        continue;
      }
      const int cb = s_cnt[cur][lb];
      const int m = ca + cb < oend ? ca + cb : oend;
      if (o0 >= m) continue;
      const double* b_d = sd + lb * lcap;
      const int* b_i = si + lb * lcap;
      // co-rank of o0: the smallest i with NOT (a[i] precedes b[o0 - i - 1]); a first on ties
      int lo = o0 > cb ? o0 - cb : 0, hi = o0 < ca ? o0 : ca;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const int j = o0 - mid - 1;
        if (!dmlp::key_less(b_d[j], b_i[j], ad[mid], ai[mid])) lo = mid + 1; else hi = mid;
      }
      int i = lo, j = o0 - lo;
      double xa = i < ca ? ad[i] : 0.0, xb = j < cb ? b_d[j] : 0.0;
      int ia = i < ca ? ai[i] : 0, ib = j < cb ? b_i[j] : 0;
      for (int o = o0; o < m; ++o) {
        const bool take_a = i < ca && (j >= cb || !dmlp::key_less(xb, ib, xa, ia));
        if (take_a) {
          od[o] = xa; oi[o] = ia;
          if (++i < ca) { xa = ad[i]; ia = ai[i]; }
        } else {
          od[o] = xb; oi[o] = ib;
          if (++j < cb) { xb = b_d[j]; ib = b_i[j]; }
        }
      }
    }
    if (lane < Ln) {
      const int la = 2 * lane, lb = la + 1;
      const int c = s_cnt[cur][la] + (lb < Lc ? s_cnt[cur][lb] : 0);
      s_cnt[cur ^ 1][lane] = c < k ? c : k;
    }
    dmlp::wave_sync();
    cur ^= 1;
    Lc = Ln;
  }
  const int total = s_cnt[cur][0];
  for (int o = lane; o < k; o += 64) {
    const bool real = o < total;
    out_d[(int64_t)q * kout + o] = real ? bd[cur][o] : INFINITY;
    out_i[(int64_t)q * kout + o] = real ? bi[cur][o] : -1;
  }
}

// Register-resident sequential form for few lists (L <= 8): one LANE per query, the L list
// heads in registers, one output per iteration (the smallest head under (dist asc, id desc);
// equal keys go to the lower list index: a later list must be strictly smaller to win), then
// one load refills the list it came from.  No LDS, no co-rank searches, no wave-wide
// synchronisation: 64 queries per wave, and the per-query work is k selections of L heads —
// the merge-path kernel spends a whole wave per query.  Padding entries (id < 0) end a list;
// slots [total, kout) get the (+inf, -1) padding, so callers need no fill pass.
template <int L>
__global__ __launch_bounds__(256) void k_merge_seq(const double* __restrict__ in_d,
                                                  const int* __restrict__ in_i,
                                                  int64_t list_stride, int kin,
                                                  const int* __restrict__ qk, int nq,
                                                  double* __restrict__ out_d,
                                                  int* __restrict__ out_i, int kout) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  int k = qk[q];
  k = k < kout ? k : kout;
  k = k > 0 ? k : 0;
  const int lim = k < kin ? k : kin;
  const int64_t qo = (int64_t)q * kin;
  double hd[L];
  int hi[L], pos[L];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    pos[l] = 0;
    hd[l] = INFINITY;
    hi[l] = -1;
    if (lim > 0) {
      hd[l] = in_d[l * list_stride + qo];
      hi[l] = in_i[l * list_stride + qo];
    }
  }
  double* const od = out_d + (int64_t)q * kout;
  int* const oi = out_i + (int64_t)q * kout;
  int o = 0;
  for (; o < k; ++o) {
    int b = -1;
    double bd = INFINITY;
    int bi = -1;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const bool better = hi[l] >= 0 && (b < 0 || dmlp::key_less(hd[l], hi[l], bd, bi));
      b = better ? l : b;
      bd = better ? hd[l] : bd;
      bi = better ? hi[l] : bi;
    }
    if (b < 0) break;  // every list exhausted
    od[o] = bd;
    oi[o] = bi;
    int pb = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) pb = l == b ? pos[l] : pb;
    ++pb;
    double nd = INFINITY;
    int ni = -1;
    if (pb < lim) {
      const int64_t off = b * list_stride + qo + pb;
      nd = in_d[off];
      ni = in_i[off];
    }
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const bool t = l == b;
      pos[l] = t ? pb : pos[l];
      hd[l] = t ? nd : hd[l];
      hi[l] = t ? ni : hi[l];
    }
  }
  for (; o < kout; ++o) {
    od[o] = INFINITY;
    oi[o] = -1;
  }
}

// Windowed form of k_merge_seq for lists whose length is a multiple of 4 (16-byte aligned
// rows): each list's next 4 entries sit in registers as a shift window (the head is always
// slot 0), filled by one 32-byte + one 16-byte load per list up front and refilled only when a
// list has given 4 outputs.  For k = 16 over 8 lists most queries never refill, so the per-lane
// chain of dependent loads (one per output in k_merge_seq) collapses to the initial fill, and
// the cache-line requests drop by 3/4 (4 entries per request instead of 1).
template <int L>
__global__ __launch_bounds__(256) void k_merge_win(const double* __restrict__ in_d,
                                                  const int* __restrict__ in_i,
                                                  int64_t list_stride, int kin,
                                                  const int* __restrict__ qk, int nq,
                                                  double* __restrict__ out_d,
                                                  int* __restrict__ out_i, int kout) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  int k = qk[q];
  k = k < kout ? k : kout;
  k = k > 0 ? k : 0;
  const int lim = k < kin ? k : kin;
  const int64_t qo = (int64_t)q * kin;
  double wd[L][4];
  int wi[L][4];
  int nxt[L];  // list position of the entry after the window
  auto fill = [&](int l, int p, double (&d)[4], int (&id)[4]) __attribute__((always_inline)) {
    const int64_t off = l * list_stride + qo + p;
    const double2 a = *(const double2*)(in_d + off);
    const double2 b = *(const double2*)(in_d + off + 2);
    const int4 c = *(const int4*)(in_i + off);
    d[0] = a.x; d[1] = a.y; d[2] = b.x; d[3] = b.y;
    // entries at or past lim end the list (the id < 0 test below)
    id[0] = p < lim ? c.x : -1;
    id[1] = p + 1 < lim ? c.y : -1;
    id[2] = p + 2 < lim ? c.z : -1;
    id[3] = p + 3 < lim ? c.w : -1;
  };
#pragma unroll
  for (int l = 0; l < L; ++l) {
    nxt[l] = 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) { wd[l][j] = INFINITY; wi[l][j] = -1; }
    if (lim > 0) fill(l, 0, wd[l], wi[l]);
  }
  double* const od = out_d + (int64_t)q * kout;
  int* const oi = out_i + (int64_t)q * kout;
  int o = 0;
  for (; o < k; ++o) {
    int b = -1;
    double bd = INFINITY;
    int bi = -1;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const bool better = wi[l][0] >= 0 && (b < 0 || dmlp::key_less(wd[l][0], wi[l][0], bd, bi));
      b = better ? l : b;
      bd = better ? wd[l][0] : bd;
      bi = better ? wi[l][0] : bi;
    }
    if (b < 0) break;  // every list exhausted
    od[o] = bd;
    oi[o] = bi;
    // shift list b's window; refill it when its last entry was just taken
    bool refill = false;
    int rp = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      if (l == b) {
        wd[l][0] = wd[l][1]; wd[l][1] = wd[l][2]; wd[l][2] = wd[l][3]; wd[l][3] = INFINITY;
        wi[l][0] = wi[l][1]; wi[l][1] = wi[l][2]; wi[l][2] = wi[l][3]; wi[l][3] = -1;
        refill = wi[l][0] < 0 && nxt[l] < lim;
        rp = nxt[l];
      }
    }
    if (refill) {
      double nd[4];
      int ni[4];
      fill(b, rp, nd, ni);
#pragma unroll
      for (int l = 0; l < L; ++l) {
        if (l == b) {
#pragma unroll
          for (int j = 0; j < 4; ++j) { wd[l][j] = nd[j]; wi[l][j] = ni[j]; }
          nxt[l] += 4;
        }
      }
    }
  }
  for (; o < kout; ++o) {
    od[o] = INFINITY;
    oi[o] = -1;
  }
}

__global__ __launch_bounds__(256) void k_finalize(const double* __restrict__ d,
                                                  const int* __restrict__ ids, int kstride,
                                                  const int* __restrict__ qk,
                                                  const int* __restrict__ qidx, int nq,
                                                  const int* __restrict__ labels, int label_lo,
                                                  int label_hi, int* __restrict__ out_label,
                                                  uint64_t* __restrict__ out_cs) {
  __shared__ int s_hist[4][kHistCap];
  const int wave = threadIdx.x >> 6;
  const int i = blockIdx.x * 4 + wave;
  if (i >= nq) return;
  const int q = qidx ? qidx[i] : i;
  const int k = qk[q];
  finalize_wave(ids + (int64_t)q * kstride, k, labels, label_lo, label_hi, s_hist[wave],
                out_label + q, out_cs + q);
}

// 64 queries x 64 points per 256-thread block; each thread a 4x4 micro-tile; attributes staged
// through LDS in chunks of 16 and accumulated strictly in attribute order.
__global__ __launch_bounds__(256) void k_exact_rows(const double* __restrict__ X, int64_t N, int A,
                                                    const double* __restrict__ Qx,
                                                    const int* __restrict__ qidx, int nq,
                                                    double* __restrict__ D, int64_t ldd) {
  constexpr int AC = 16;
  __shared__ double Qs[64][AC + 1];
  __shared__ double Xs[64][AC + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t pt0 = (int64_t)blockIdx.x * 64;
  const int qt0 = blockIdx.y * 64;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  for (int a0 = 0; a0 < A; a0 += AC) {
    const int ac = A - a0 < AC ? A - a0 : AC;
    for (int e = tid; e < 64 * AC; e += 256) {
      const int r = e / AC, a = e % AC;
      const int qi = qt0 + r;
      Qs[r][a] = (qi < nq && a < ac) ? Qx[(int64_t)qidx[qi] * A + a0 + a] : 0.0;
      const int64_t pi = pt0 + r;
      Xs[r][a] = (pi < N && a < ac) ? X[pi * A + a0 + a] : 0.0;
    }
    __syncthreads();
    for (int a = 0; a < ac; ++a) {
      double qv[4], xv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) qv[i] = Qs[ty + 16 * i][a];
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[j] = Xs[tx + 16 * j][a];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double dd = __dsub_rn(qv[i], xv[j]);
          acc[i][j] = __dadd_rn(acc[i][j], __dmul_rn(dd, dd));
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qi = qt0 + ty + 16 * i;
    if (qi >= nq) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t pi = pt0 + tx + 16 * j;
      if (pi < N) D[(int64_t)qi * ldd + pi] = acc[i][j];
    }
  }
}

// ---- report formatting: "Query <qid> checksum: <cs>\n"
__device__ __forceinline__ int ndig_u64(uint64_t v) {
  int n = 1;
  while (v >= 10) { v /= 10; ++n; }
  return n;
}
__device__ __forceinline__ int line_len(int64_t qid, uint64_t cs) {
  return 6 + ndig_u64((uint64_t)qid) + 11 + ndig_u64(cs) + 1;
}

template <int FB>
__global__ void __launch_bounds__(FB) k_fmt_len(const uint64_t* __restrict__ cs, int nq,
                                                int qid_base, int64_t* __restrict__ off,
                                                int64_t* __restrict__ blocksum) {
  __shared__ int64_t sh[FB];
  const int i = blockIdx.x * FB + threadIdx.x;
  const int64_t v = i < nq ? line_len((int64_t)qid_base + i, cs[i]) : 0;
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int o = 1; o < FB; o <<= 1) {  // inclusive Hillis-Steele scan
    const int64_t t = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  if (i < nq) off[i + 1] = sh[threadIdx.x];  // block-local inclusive
  if (threadIdx.x == FB - 1) blocksum[blockIdx.x] = sh[FB - 1];
}

// Exclusive scan of the block sums in place (+ the total at [nb]): one 1024-thread block,
// 1024 sums per LDS pass with a running carry (a single-thread loop cost ~15 us at 128 blocks —
// one dependent global round trip per block).
__global__ void __launch_bounds__(1024) k_fmt_scan_blocks(int64_t* __restrict__ blocksum, int nb) {
  __shared__ int64_t sh[1024];
  int64_t carry = 0;
  for (int c0 = 0; c0 < nb; c0 += 1024) {
    const int b = c0 + (int)threadIdx.x;
    const int64_t v = b < nb ? blocksum[b] : 0;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
      const int64_t t = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0;
      __syncthreads();
      sh[threadIdx.x] += t;
      __syncthreads();
    }
    if (b < nb) blocksum[b] = carry + sh[threadIdx.x] - v;  // exclusive
    carry += sh[1023];
    __syncthreads();  // sh is rewritten by the next pass
  }
  if (threadIdx.x == 0) blocksum[nb] = carry;
}

// decimal digits of v written backwards so that the last one lands at txt[end - 1]: two 64-bit
// divisions by 1e9 at most, then 32-bit digit extraction (no per-digit 64-bit division, no
// dynamically indexed scratch buffer)
__device__ __forceinline__ void put_dec(char* txt, int end, uint64_t v) {
  int p = end;
  while (v >= 1000000000ull) {
    const uint64_t q = v / 1000000000ull;
    uint32_t r = (uint32_t)(v - q * 1000000000ull);
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      txt[--p] = (char)('0' + r % 10u);
      r /= 10u;
    }
    v = q;
  }
  uint32_t r = (uint32_t)v;
  do {
    txt[--p] = (char)('0' + r % 10u);
    r /= 10u;
  } while (r);
}

// Each block renders its FB lines into LDS, then stores the block's byte range with dword
// stores (bytes only at the two unaligned ends).  The target may be page-locked host memory
// (the native engine writes the report straight into its output buffer): wide, contiguous
// stores keep the link busy where per-character stores would not.
template <int FB>
__global__ void __launch_bounds__(FB) k_fmt_write(const uint64_t* __restrict__ cs, int nq,
                                                 int qid_base, int64_t* __restrict__ off,
                                                 const int64_t* __restrict__ blocksum,
                                                 const int64_t* __restrict__ base,
                                                 char* __restrict__ out) {
  __shared__ char txt[FB * 48 + 4];
  const int i = blockIdx.x * FB + threadIdx.x;
  const int64_t b0 = base ? *base : 0;  // byte offset of this run's first line in out
  const int64_t g0 = b0 + blocksum[blockIdx.x], g1 = b0 + blocksum[blockIdx.x + 1];
  if (i < nq) {
    const int64_t qid = (int64_t)qid_base + i;
    const uint64_t v = cs[i];
    const int len = line_len(qid, v);
    const int64_t endl = off[i + 1];  // block-local inclusive end
    int pos = (int)(endl - len);
    const char* pre = "Query ";
    for (int c = 0; c < 6; ++c) txt[pos++] = pre[c];
    pos += ndig_u64((uint64_t)qid);
    put_dec(txt, pos, (uint64_t)qid);
    const char* mid = " checksum: ";
    for (int c = 0; c < 11; ++c) txt[pos++] = mid[c];
    pos += ndig_u64(v);
    put_dec(txt, pos, v);
    txt[pos++] = '\n';
  }
  __syncthreads();
  const int64_t a0 = (g0 + 3) & ~int64_t(3), a1 = std::max(a0, g1 & ~int64_t(3));
  if (threadIdx.x < 3) {  // unaligned head / tail bytes
    const int64_t h = g0 + threadIdx.x, tl = a1 + threadIdx.x;
    if (h < a0 && h < g1) out[h] = txt[h - g0];
    if (tl < g1 && tl >= a0) out[tl] = txt[tl - g0];
  }
  unsigned* o32 = reinterpret_cast<unsigned*>(out + a0);
  const int nw = (int)((a1 - a0) >> 2), b = (int)(a0 - g0);
  for (int w = threadIdx.x; w < nw; w += FB) {
    const int s = b + 4 * w;
    o32[w] = (unsigned)(unsigned char)txt[s] | ((unsigned)(unsigned char)txt[s + 1] << 8) |
             ((unsigned)(unsigned char)txt[s + 2] << 16) |
             ((unsigned)(unsigned char)txt[s + 3] << 24);
  }
  if (i < nq) off[i + 1] += g0;
  if (i == 0) off[0] = b0;
}


// element i of a row table: the fp64 rows, or (Xi non-null) the lossless int32 rows divided back
// exactly as k_rows_from_i32 does (prep.hip: the host checked x == fl(m / 1e6) for every value)
__device__ __forceinline__ double row_value(const double* __restrict__ X, const int* __restrict__ Xi,
                                            int64_t i) {
  return Xi ? (double)Xi[i] / 1.0e6 : X[i];
}

// Group refine, TWO queries per wave (32 lanes each): the one-slice single-term screen on the
// host's fp16 operands (S = 1, hl = 1, KT <= 2), k <= 64, labels given.  k_refine (one query per
// wave) is bound by its chain of dependent gathers — group entries -> member fragments -> exact
// rows -> labels — at 8 waves per SIMD, i.e. 8 queries in flight per SIMD; here each wave keeps
// two queries' chains in flight with about the same registers per lane.  Members are scored two
// per lane per batch (64 per query), so the usual ~72 members take 2 batches.  More than PM
// surviving members hand the query back (status 1, as k_refine does past its P).
#ifndef DMLP_PAIR_U
#define DMLP_PAIR_U 1  // members per lane per batch (1 at 8 waves/SIMD: 239 us vs 289 us for 2 at 5, r7w)
#endif
constexpr int PAIR_U = DMLP_PAIR_U;
#ifndef DMLP_PAIR_RL
#define DMLP_PAIR_RL 8  // lanes per exact row in the survivors' phase: 8 (218 us), 16 (239 us, r8c) or 4 (222 us, r12p)
#endif
#ifndef DMLP_PAIR_DOT2
#define DMLP_PAIR_DOT2 1  // member scores by v_dot2c_f32_f16 (219 -> 212 us, 0 spills; r8h) or cvt + fma
#endif
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
#ifndef DMLP_PAIR_WPE
#define DMLP_PAIR_WPE 8  // (U = 2: 5, 288 us; profiles/r7n_refine_ab.txt)
#endif
template <int KT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KT == 1 ? DMLP_PAIR_WPE : 4))) void k_refine_pair(
    const int* __restrict__ cand_ids, const int* __restrict__ cand_cnt, int cap,
    const float* __restrict__ cand_h, const double* __restrict__ X, int A,
    const double* __restrict__ Qx, const int* __restrict__ Xi, const int* __restrict__ Qi,
    const int* __restrict__ qidx, const int* __restrict__ qk,
    int nq, const u32x4* __restrict__ xfrag, const u32x4* __restrict__ xrow,
    const float* __restrict__ xinit, const bf16x8* __restrict__ qhi, int n_points,
    double* __restrict__ out_d, int* __restrict__ out_i, int kstride,
    const int* __restrict__ labels, int* __restrict__ out_label, uint64_t* __restrict__ out_cs,
    int* __restrict__ status, int* __restrict__ ovf_count, int abl, int grows) {
  constexpr int PM = 64;   // surviving members per query
  constexpr int KM = 64;   // k
  constexpr int EC = 4;    // group entries held per lane (cap <= 128)
  __shared__ int s_i[8][PM];
  __shared__ double s_d[8][PM];
  __shared__ int s_l[8][PM];
  __shared__ double s_rd[8][KM];
  __shared__ int s_ri[8][KM];
  __shared__ int s_rl[8][KM];
#if DMLP_PAIR_DOT2
  __shared__ __attribute__((aligned(16))) unsigned s_qh[8][16 * KT];  // hi(q') as fp16 pairs
#else
  __shared__ __attribute__((aligned(16))) float s_qf[8][32 * KT];  // hi(q') as fp32
#endif
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int half = lane >> 5, hl = lane & 31;
  const int slot = wave * 2 + half;
  const int p = blockIdx.x * 8 + slot;
  bool act = p < nq;
  const int q = act ? (qidx ? qidx[p] : p) : 0;
  const int k = act ? qk[q] : 0;
  const int n = act ? cand_cnt[p] : 0;
  const float hq = act ? cand_h[2 * (int64_t)p] : 0.0f;
  unsigned ent[EC];
#pragma unroll
  for (int u = 0; u < EC; ++u) {
    const int j = hl + 32 * u;
    ent[u] = act && j < n && j < cap ? (unsigned)cand_ids[(int64_t)p * cap + j] : 0u;
  }
  // hi(q') as fp32 in LDS, read at each use (held in registers it pushed the kernel into spills)
  {
    const unsigned short* qh = (const unsigned short*)(qhi + (int64_t)q * KT * 4);
#if DMLP_PAIR_DOT2
    for (int a = hl; a < 16 * KT; a += 32)
      s_qh[slot][a] = act ? (unsigned)qh[2 * a] | ((unsigned)qh[2 * a + 1] << 16) : 0u;
#else
    for (int a = hl; a < 32 * KT; a += 32)
      s_qf[slot][a] = act ? (float)__builtin_bit_cast(_Float16, qh[a]) : 0.0f;
#endif
  }
  if (act)
    for (int i = k + hl; i < kstride; i += 32) {
      out_d[(int64_t)q * kstride + i] = INFINITY;
      out_i[(int64_t)q * kstride + i] = -1;
    }
  if (act && n < 0) {
    if (hl == 0) {
      status[q] = 1;
      atomicAdd(ovf_count, 1);
    }
    act = false;
  } else if (act && hl == 0) {
    status[q] = 0;
  }
  const int M = act ? n : 0;
  const unsigned tq = __float_as_uint(hq);
  const unsigned kh = (tq ^ ((unsigned)((int)tq >> 31) | 0x80000000u)) & 0xffff0000u;
  // ---- members: two per lane per batch; keep those whose single-term score reaches hq
  int Mw = M;  // wave-uniform trip count: the larger half's
  Mw = max(Mw, __shfl_xor(Mw, 32));
  int nm = 0;
  dmlp::wave_sync();  // s_qf written
  const int GS = grows == 8 ? 3 : 2;  // members per group entry, log2
  for (int j0 = 0; j0 < (Mw << GS); j0 += 32 * PAIR_U) {
    __asm__ volatile("" ::: "memory");  // keep the s_qf reads in the loop
    int id[PAIR_U];
    bool pass[PAIR_U];
    u32x4 w[PAIR_U][KT * 4];
    float sc[PAIR_U];
#pragma unroll
    for (int u = 0; u < PAIR_U; ++u) {
      const int jm = j0 + 32 * u + hl;
      const int g = jm >> GS;
      const int src = half * 32 + (g & 31);
      unsigned e = 0;
#pragma unroll
      for (int c = 0; c < EC; ++c) {
        const unsigned v = (unsigned)__shfl((int)ent[c], src);
        if ((g >> 5) == c) e = v;
      }
      id[u] = group_row(e & 0xffffu, jm & (grows - 1), grows);
      pass[u] = g < M && e >= kh && id[u] < n_points;
      const int pt = pass[u] ? id[u] : 0;
      if (xrow) {  // the point's 64 * KT bytes in one run (k_x1_rowmajor): one line per member
        const u32x4* fr = xrow + (int64_t)pt * (4 * KT);
#pragma unroll
        for (int f = 0; f < 4 * KT; ++f)
          w[u][f] = pass[u] && !(abl & 2) ? fr[f] : u32x4{0, 0, 0, 0};
      } else {
        const u32x4* fr = xfrag + (int64_t)(pt >> 6) * (4 * KT * 64) + (pt & 15);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
          for (int kq = 0; kq < 4; ++kq)
            w[u][kt * 4 + kq] = pass[u] && !(abl & 2) ? fr[(int64_t)((((pt & 63) >> 4) * KT + kt) * 64) + 16 * kq]
                                        : u32x4{0, 0, 0, 0};
      }
      sc[u] = pass[u] ? xinit[pt] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < PAIR_U; ++u) {
#pragma unroll
      for (int f = 0; f < KT * 4; ++f) {
#if DMLP_PAIR_DOT2
        // v_dot2c_f32_f16: two exact fp16 products added into the fp32 score per instruction (at
        // most two roundings per pair, A in all: inside the screen bound like the MFMA's chain;
        // fp16 subnormal inputs are not flushed: tools/probe/dot2_probe.hip).  The words are taken
        // out of the vectors first: w[u][f][q2] inside the builtin's operand compiled to word 0
        // of each fragment for every q2 (one dword load per fragment, wrong scores)
        const uint4 qv = *(const uint4*)&s_qh[slot][4 * f];
        const u32x4 xv = w[u][f];
        const unsigned qw[4] = {qv.x, qv.y, qv.z, qv.w};
        const unsigned xw[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2)
          sc[u] = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2v, qw[q2]),
                                         __builtin_bit_cast(f16x2v, xw[q2]), sc[u], false);
#else
        const float4 q0 = *(const float4*)&s_qf[slot][8 * f];
        const float4 q1 = *(const float4*)&s_qf[slot][8 * f + 4];
        const float qf[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          const unsigned xw = w[u][f][q2];
          // fp16 x fp16 products are exact in fp32: fma == multiply-then-add here
          sc[u] = __builtin_fmaf(qf[2 * q2], (float)__builtin_bit_cast(_Float16, (unsigned short)(xw & 0xffffu)), sc[u]);
          sc[u] = __builtin_fmaf(qf[2 * q2 + 1], (float)__builtin_bit_cast(_Float16, (unsigned short)(xw >> 16)), sc[u]);
        }
#endif
      }
      const bool keep = pass[u] && sc[u] >= hq;
      const unsigned long long bm = __ballot(keep);
      const unsigned hm = (unsigned)(bm >> (32 * half));
      const int pos = nm + __popc(hm & ((1u << hl) - 1u));
      if (keep && pos < PM) s_i[slot][pos] = id[u];
      nm += __popc(hm);
    }
  }
  if (act && nm > PM) {  // pathological ties: hand the query back
    if (hl == 0) {
      status[q] = 1;
      atomicAdd(ovf_count, 1);
    }
    act = false;
  }
  const int Ms = act ? nm : 0;
  dmlp::wave_sync();
  // ---- exact distances of the survivors in the reference's order (engine.cpp:12-18), 16 lanes
  // per row: lane t loads attributes 2t, 2t+1 (+ 32 u) of the row — one row is two cache lines
  // read by one instruction, where a lane-per-row gather touched a line per lane per load (the
  // rows were half of this kernel's time: profiles/r7m_refine_ablation.txt) — squares their
  // differences (each product rounded, no FMA), and the left-to-right sum travels from lane to
  // lane by a DPP row rotate, so lane 15 ends with exactly the reference's sum.
#if DMLP_PAIR_RL == 16
  {
    const int t16 = hl & 15, rsel = hl >> 4;
    double qa[KT][2];
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int a0 = 32 * u + 2 * t16;
      qa[u][0] = a0 < A ? row_value(Qx, Qi, (int64_t)q * A + a0) : 0.0;
      qa[u][1] = a0 + 1 < A ? row_value(Qx, Qi, (int64_t)q * A + a0 + 1) : 0.0;
    }
    int Msw = Ms;
    Msw = max(Msw, __shfl_xor(Msw, 32));
    for (int r0 = 0; r0 < Msw; r0 += 2) {
      const int j = r0 + rsel;
      const bool rv = j < Ms;
      const int id = rv ? s_i[slot][j] : 0;
      const int64_t xb = (int64_t)id * A;
      double pr[KT][2];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const int a0 = 32 * u + 2 * t16;
        const double x0 = rv && a0 < A && !(abl & 1) ? row_value(X, Xi, xb + a0) : 0.0;
        const double x1 = rv && a0 + 1 < A && !(abl & 1) ? row_value(X, Xi, xb + a0 + 1) : 0.0;
        const double d0 = a0 < A ? __dsub_rn(qa[u][0], x0) : 0.0;
        const double d1 = a0 + 1 < A ? __dsub_rn(qa[u][1], x1) : 0.0;
        pr[u][0] = __dmul_rn(d0, d0);
        pr[u][1] = __dmul_rn(d1, d1);
      }
      double sm = 0.0;
#pragma unroll
      for (int u = 0; u < KT; ++u)
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          // lane t's turn: its predecessor's partial sum arrives by the rotate (lane 0 gets lane
          // 15's: 0 at the start, the previous 32-attribute chunk's total after it)
          const long long b = __double_as_longlong(sm);
          const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x121, 0xf, 0xf, false);
          const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x121, 0xf, 0xf, false);
          const double in = __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
          sm = t16 == t ? __dadd_rn(__dadd_rn(in, pr[u][0]), pr[u][1]) : sm;
        }
      if (rv && t16 == 15) {
        s_d[slot][j] = (abl & 1) ? (double)id : sm;
        s_l[slot][j] = labels[id];
      }
    }
  }
#else
  // 8 lanes per row (four rows per round; DMLP_PAIR_RL=4: 4 lanes, eight rows): lane t holds
  // attributes E t .. E t + E-1 (+ 32 u), adds its E products to its predecessor's partial sum in
  // order, and the sum moves on by a DPP row shift — fewer rounds and chain steps than 16 lanes
  {
    constexpr int RL = DMLP_PAIR_RL, E = 32 / RL;
    const int t8 = hl & (RL - 1), rsel = hl / RL;
    double qa[KT][E];
#pragma unroll
    for (int u = 0; u < KT; ++u)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int a = 32 * u + E * t8 + e;
        qa[u][e] = a < A ? row_value(Qx, Qi, (int64_t)q * A + a) : 0.0;
      }
    int Msw = Ms;
    Msw = max(Msw, __shfl_xor(Msw, 32));
    for (int r0 = 0; r0 < Msw; r0 += 32 / RL) {
      const int j = r0 + rsel;
      const bool rv = j < Ms;
      const int id = rv ? s_i[slot][j] : 0;
      const int64_t xb = (int64_t)id * A;
      double pr[KT][E];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const int a0 = 32 * u + E * t8;
        double x[E];
        if (Xi && rv && !(abl & 1) && a0 + E - 1 < A && (A & 3) == 0 && E % 4 == 0) {
          // lossless int32 rows: half the bytes of the gather (one 16-byte load per 4 values),
          // each value divided back exactly as k_rows_from_i32 does
#pragma unroll
          for (int e = 0; e < E; e += 4) {
            const int4 v = *(const int4*)(Xi + xb + a0 + e);
            x[e] = (double)v.x / 1.0e6;
            x[e + 1] = (double)v.y / 1.0e6;
            x[e + 2] = (double)v.z / 1.0e6;
            x[e + 3] = (double)v.w / 1.0e6;
          }
        } else if (!Xi && rv && !(abl & 1) && a0 + E - 1 < A && (A & 1) == 0) {  // 16-byte pairs
#pragma unroll
          for (int e = 0; e < E; e += 2) {
            const double2 v = *(const double2*)(X + xb + a0 + e);
            x[e] = v.x;
            x[e + 1] = v.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e)
            x[e] = rv && !(abl & 1) && a0 + e < A ? row_value(X, Xi, xb + a0 + e) : 0.0;
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const double d = a0 + e < A ? __dsub_rn(qa[u][e], x[e]) : 0.0;
          pr[u][e] = __dmul_rn(d, d);
        }
      }
      double sm = 0.0;
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        // lane 0 of the group continues from the last lane's total of the previous 32 attributes
        const double tl = u == 0 ? 0.0 : __shfl(sm, (lane & ~(RL - 1)) | (RL - 1));
#pragma unroll
        for (int t = 0; t < RL; ++t) {
          double in = tl;
          if (t > 0) {
            const long long b = __double_as_longlong(sm);
            const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x111, 0xf, 0xf, false);
            const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x111, 0xf, 0xf, false);
            in = __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
          }
          double v = in;
#pragma unroll
          for (int e = 0; e < E; ++e) v = __dadd_rn(v, pr[u][e]);
          sm = t8 == t ? v : sm;
        }
      }
      if (rv && t8 == RL - 1) {
        s_d[slot][j] = (abl & 1) ? (double)id : sm;
        s_l[slot][j] = labels[id];
      }
    }
  }
#endif
  for (int i = hl; i < KM; i += 32) {
    s_rd[slot][i] = INFINITY;
    s_ri[slot][i] = -1;
    s_rl[slot][i] = 0;
  }
  dmlp::wave_sync();
  // ---- rank select: keys are unique, rank = #{ keys before } places the top-k directly
  for (int j = hl; j < Ms; j += 32) {
    const double dj = s_d[slot][j];
    const int ij = s_i[slot][j];
    int r = 0;
    for (int i = 0; i < Ms; ++i) r += dmlp::key_less(s_d[slot][i], s_i[slot][i], dj, ij) ? 1 : 0;
    if (r < k) {
      s_rd[slot][r] = dj;
      s_ri[slot][r] = ij;
      s_rl[slot][r] = s_l[slot][j];
    }
  }
  dmlp::wave_sync();
  if (act)
    for (int i = hl; i < k; i += 32) {
      out_d[(int64_t)q * kstride + i] = s_rd[slot][i];
      out_i[(int64_t)q * kstride + i] = s_ri[slot][i];
    }
  // ---- vote (max count, tie -> larger label; padding ids < 0 not counted) + FNV checksum
  long long best = -1;
  for (int i = hl; i < k; i += 32) {
    if (s_ri[slot][i] < 0) continue;
    const int li = s_rl[slot][i];
    int c = 0;
    for (int j = 0; j < k; ++j) c += (s_ri[slot][j] >= 0 && s_rl[slot][j] == li) ? 1 : 0;
    const long long key = ((long long)c << 32) | (long long)((unsigned)li ^ 0x80000000u);
    best = key > best ? key : best;
  }
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) {
    const long long o = __shfl_xor(best, off);
    best = o > best ? o : best;
  }
  if (act && hl == 0) {
    const int label = best < 0 ? -1 : (int)((unsigned)(best & 0xffffffffll) ^ 0x80000000u);
    out_label[q] = label;
    out_cs[q] = dmlp::fnv_checksum(label, s_ri[slot], k);
  }
}

}  // namespace

extern "C" int dmlp_refine(int cap, const int* cand_ids, const int* cand_cnt, int S,
                           const double* X, int A, const double* Qx, const int* qidx,
                           const int* qk, int nq, double* out_d, int* out_i, int kstride,
                           const int* labels, int label_lo, int label_hi, int* out_label,
                           uint64_t* out_cs, int* status, int* ovf_count, void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || S > 256) return -1;
  const dim3 grid((nq + 3) / 4), block(256);
  hipStream_t st = (hipStream_t)stream;
  // cap is only the id stride per (query, slice).  P = 256 slots cover k + 64 for every k of the
  // cap <= 256 screens (<= 128); a larger P would cut the resident waves that hide the
  // row-gather latency, so only the cap-512 screen (128 < k <= 256) takes P = 512
  if (cap < 1) return -2;
  if (cap > 256)
    hipLaunchKernelGGL((k_refine<8, 0>), grid, block, 0, st, cand_ids, cand_cnt, S, cap, X, A,
                       Qx, qidx, qk, nq, out_d, out_i, kstride, labels, label_lo, label_hi,
                       out_label, out_cs, status, ovf_count, GroupIn{});
  else
    hipLaunchKernelGGL((k_refine<4, 0>), grid, block, 0, st, cand_ids, cand_cnt, S, cap, X, A,
                       Qx, qidx, qk, nq, out_d, out_i, kstride, labels, label_lo, label_hi,
                       out_label, out_cs, status, ovf_count, GroupIn{});
  DMLP_LAUNCH_CHECK();
  return 0;
}

static int refine_groups_impl(int cap, const int* cand_ids, const int* cand_cnt,
                              const float* cand_h, int S, const double* X, int A, const double* Qx,
                              const void* xfrag, const void* xrow, const float* xinit,
                              const void* qhi, int KT, int hl, int64_t n_points, const int* qidx,
                              const int* qk, int nq, double* out_d, int* out_i, int kstride,
                              const int* labels, int label_lo, int label_hi, int* out_label,
                              uint64_t* out_cs, int* status, int* ovf_count, int collect,
                              void* stream, int kmax = 64, int grows = 4,
                              const int* Xi = nullptr, const int* Qi = nullptr) {
  if (nq <= 0) return 0;
  if (grows != 4 && grows != 8) return -1;
  if (S < 1 || S > 256 || cap < 1 || n_points > 0x7fffffff) return -1;
  if (KT != 1 && KT != 2 && KT != 4 && KT != 8) return -1;
  if (hl != 1 && hl != 2) return -1;
  const int64_t n_tiles = (n_points + 63) / 64;
  GroupIn gin{cand_h, (const u32x4*)xfrag, xinit, (const bf16x8*)qhi, KT, hl, (int)n_points,
              (int)((n_tiles + S - 1) / S), collect ? 1 : 0};
  gin.grows = collect ? 4 : grows;
  gin.xi32 = Xi;
  // collect (the large-k lists, fp16 host operands only): k <= 256 over <= 512 filtered members
  if (collect) {
    if (hl != 1) return -1;
#define DMLP_REFINE_GB(KTV)                                                                    \
  hipLaunchKernelGGL((k_refine<8, KTV, true>), dim3((nq + 3) / 4), dim3(256), 0, (hipStream_t)stream, \
                     cand_ids, cand_cnt, S, cap, X, A, Qx, qidx, qk, nq, out_d, out_i, kstride, \
                     labels, label_lo, label_hi, out_label, out_cs, status, ovf_count, gin)
    if (KT == 1) DMLP_REFINE_GB(1);
    else if (KT == 2) DMLP_REFINE_GB(2);
    else if (KT == 4) DMLP_REFINE_GB(4);
    else DMLP_REFINE_GB(8);
#undef DMLP_REFINE_GB
    DMLP_LAUNCH_CHECK();
    return 0;
  }
  // one slice of the host's fp16 operands, k <= 32, labels: two queries per wave
  // (k_refine_pair; DMLP_REFINE_PAIR=0: the one-query-per-wave kernel).  Its PM = 64 member slots
  // leave >= 32 of slack above k only for k <= 32: at k near 64 any member inside the 2-eps band
  // would hand the query back, so the class k in (32, 64] takes k_refine (P = 128 slots)
  // DMLP_REFINE_ABL (timing ablations, wrong results): 1 no exact-row gathers, 2 no member loads
  static const int pair_abl = getenv("DMLP_REFINE_ABL") ? atoi(getenv("DMLP_REFINE_ABL")) : 0;
  if (dmlp_refine_pair_path(S, hl, KT, labels != nullptr, cap, kmax)) {
    const dim3 grid((unsigned)((nq + 7) / 8));
    if (KT == 1)
      hipLaunchKernelGGL((k_refine_pair<1>), grid, dim3(256), 0, (hipStream_t)stream, cand_ids,
                         cand_cnt, cap, cand_h, X, A, Qx, Xi, Qi, qidx, qk, nq, (const u32x4*)xfrag,
                         (const u32x4*)xrow, xinit, (const bf16x8*)qhi, (int)n_points, out_d, out_i,
                         kstride, labels, out_label,
                         out_cs, status, ovf_count, pair_abl, gin.grows);
    else
      hipLaunchKernelGGL((k_refine_pair<2>), grid, dim3(256), 0, (hipStream_t)stream, cand_ids,
                         cand_cnt, cap, cand_h, X, A, Qx, Xi, Qi, qidx, qk, nq, (const u32x4*)xfrag,
                         (const u32x4*)xrow, xinit, (const bf16x8*)qhi, (int)n_points, out_d, out_i,
                         kstride, labels, out_label,
                         out_cs, status, ovf_count, pair_abl, gin.grows);
    DMLP_LAUNCH_CHECK();
    return 0;
  }
  if ((!X && !Xi) || !Qx) return -3;  // (the other refines read fp64 queries)
#define DMLP_REFINE_G(KTV, F16)                                                                \
  hipLaunchKernelGGL((k_refine<2, KTV, F16>), dim3((nq + 3) / 4), dim3(256), 0, (hipStream_t)stream, \
                     cand_ids, cand_cnt, S, cap, X, A, Qx, qidx, qk, nq, out_d, out_i, kstride, \
                     labels, label_lo, label_hi, out_label, out_cs, status, ovf_count, gin)
  if (KT == 1) {
    if (hl == 1) DMLP_REFINE_G(1, true);
    else DMLP_REFINE_G(1, false);
  } else if (KT == 2) {
    if (hl == 1) DMLP_REFINE_G(2, true);
    else DMLP_REFINE_G(2, false);
  } else if (KT == 4) {
    if (hl == 1) DMLP_REFINE_G(4, true);
    else DMLP_REFINE_G(4, false);
  } else {
    if (hl == 1) DMLP_REFINE_G(8, true);
    else DMLP_REFINE_G(8, false);
  }
#undef DMLP_REFINE_G
  DMLP_LAUNCH_CHECK();
  return 0;
}

// The exact path's fp64 screen (screen_f64.hip): group ids of 4-point groups in slices of
// tiles_per_slice 64-point tiles, no rescoring image — every member of a group at or above the
// global threshold is re-ranked exactly (<= 512 members, k <= 256: the E = 8 variant).  Writes
// out_d / out_i only (no vote).
extern "C" int dmlp_refine_groups_exact(int cap, const int* cand_ids, const int* cand_cnt,
                                        const float* cand_h, int S, int64_t tiles_per_slice,
                                        const double* X, int A, const double* Qx, int64_t n_points,
                                        const int* qidx, const int* qk, int nq, double* out_d,
                                        int* out_i, int kstride, int* status, int* ovf_count,
                                        void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || S > 256 || cap < 1 || n_points > 0x7fffffff || tiles_per_slice < 1) return -1;
  GroupIn gin{cand_h, nullptr, nullptr, nullptr, 1, 1, (int)n_points, (int)tiles_per_slice, 0};
  gin.rescore = 0;
  hipLaunchKernelGGL((k_refine<8, 1, true>), dim3((nq + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     cand_ids, cand_cnt, S, cap, X, A, Qx, qidx, qk, nq, out_d, out_i, kstride,
                     nullptr, 0, 1, nullptr, nullptr, status, ovf_count, gin);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_refine_groups2(int cap, const int* cand_ids, const int* cand_cnt,
                                   const float* cand_h, int S, const double* X, int A,
                                   const double* Qx, const void* xfrag, const float* xinit,
                                   const void* qhi, int KT, int hl, int64_t n_points,
                                   const int* qidx, const int* qk, int nq, double* out_d,
                                   int* out_i, int kstride, const int* labels, int label_lo,
                                   int label_hi, int* out_label, uint64_t* out_cs, int* status,
                                   int* ovf_count, int collect, void* stream) {
  // (the lists' producer, by its cap: dmlp_screen_x1_cap(kmax) of the screen that wrote them)
  const int grows = collect ? 4 : dmlp_screen_x1_group_rows_kt(KT, 64);
  return refine_groups_impl(cap, cand_ids, cand_cnt, cand_h, S, X, A, Qx, xfrag, nullptr, xinit,
                            qhi, KT, hl, n_points, qidx, qk, nq, out_d, out_i, kstride, labels,
                            label_lo, label_hi, out_label, out_cs, status, ovf_count, collect,
                            stream, 64, grows);
}

extern "C" int dmlp_refine_groups_rm(int cap, const int* cand_ids, const int* cand_cnt,
                                     const float* cand_h, int S, const double* X, int A,
                                     const double* Qx, const void* xfrag, const void* xrow,
                                     const float* xinit, const void* qhi, int KT, int hl,
                                     int64_t n_points, const int* qidx, const int* qk, int nq,
                                     double* out_d, int* out_i, int kstride, const int* labels,
                                     int label_lo, int label_hi, int* out_label, uint64_t* out_cs,
                                     int* status, int* ovf_count, int kmax, const int* Xi,
                                     const int* Qi, void* stream) {
  return refine_groups_impl(cap, cand_ids, cand_cnt, cand_h, S, X, A, Qx, xfrag, xrow, xinit, qhi,
                            KT, hl, n_points, qidx, qk, nq, out_d, out_i, kstride, labels,
                            label_lo, label_hi, out_label, out_cs, status, ovf_count, 0, stream,
                            kmax, dmlp_screen_x1_group_rows_kt(KT, kmax), Xi, Qi);
}

// Whether refine_groups_impl serves these lists with k_refine_pair: one slice of the host's fp16
// operands (S = 1, hl = 1, KT <= 2), labels, k <= 32 (PM = 64 member slots leave >= 32 of slack
// above k only there: at k near 64 any member inside the 2-eps band would hand the query back,
// so the class k in (32, 64] takes k_refine, P = 128 slots).  DMLP_REFINE_PAIR=0: never.  The
// pair refine also reads lossless int32 rows (dmlp_refine_groups_rm Xi / Qi), the others fp64.
extern "C" int dmlp_refine_pair_path(int S, int hl, int KT, int labels, int cap, int kmax) {
  static const bool pair_on = !(getenv("DMLP_REFINE_PAIR") && getenv("DMLP_REFINE_PAIR")[0] == '0');
  return pair_on && S == 1 && hl == 1 && KT <= 2 && labels && cap <= 128 && kmax <= 32 ? 1 : 0;
}

// The host-rendered fp16 image (tile layout of the screen's MFMA A operand: point p's 8-element
// chunk f at u32x4 index tile * 256 KT + ((p & 63) >> 4) KT 64 + (f >> 2) 64 + 16 (f & 3) +
// (p & 15)) copied point-major, xrow[p][f]: the pair refine's member loads then read one 64 KT
// byte run per member instead of 4 KT separate lines
__global__ __launch_bounds__(256) void k_x1_rowmajor(const u32x4* __restrict__ xfrag,
                                                     int64_t n_items, int KT,
                                                     u32x4* __restrict__ xrow) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // = p * 4 KT + f
  if (i >= n_items) return;
  const int nf = 4 * KT;
  const int64_t pt = i / nf;
  const int f = (int)(i - pt * nf), kt = f >> 2, kq = f & 3;
  xrow[i] = xfrag[(pt >> 6) * (4 * KT * 64) + ((((pt & 63) >> 4) * KT + kt) * 64) + 16 * kq +
                  (pt & 15)];
}

extern "C" int dmlp_x1_rowmajor(const void* xfrag, int64_t n_tiles, int KT, void* xrow,
                                void* stream) {
  if (n_tiles <= 0) return 0;
  if (KT < 1 || KT > 8) return -1;
  const int64_t n = n_tiles * 64 * 4 * KT;
  hipLaunchKernelGGL(k_x1_rowmajor, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const u32x4*)xfrag, n, KT, (u32x4*)xrow);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_refine_groups(int cap, const int* cand_ids, const int* cand_cnt,
                                  const float* cand_h, int S, const double* X, int A,
                                  const double* Qx, const void* xfrag, const float* xinit,
                                  const void* qhi, int KT, int hl, int64_t n_points, const int* qidx,
                                  const int* qk, int nq, double* out_d, int* out_i, int kstride,
                                  const int* labels, int label_lo, int label_hi, int* out_label,
                                  uint64_t* out_cs, int* status, int* ovf_count, void* stream) {
  return dmlp_refine_groups2(cap, cand_ids, cand_cnt, cand_h, S, X, A, Qx, xfrag, xinit, qhi, KT,
                             hl, n_points, qidx, qk, nq, out_d, out_i, kstride, labels, label_lo,
                             label_hi, out_label, out_cs, status, ovf_count, 0, stream);
}

extern "C" int dmlp_exact_rows(const double* X, int64_t N, int A, const double* Qx,
                               const int* qidx, int nq, double* D, int64_t ldd, void* stream) {
  if (nq <= 0 || N <= 0) return 0;
  const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((nq + 63) / 64));
  hipLaunchKernelGGL(k_exact_rows, grid, dim3(256), 0, (hipStream_t)stream, X, N, A, Qx, qidx,
                     nq, D, ldd);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_merge(const double* in_d, const int* in_i, int L, int64_t list_stride,
                          int kin, const int* qk, int nq, double* out_d, int* out_i, int kout,
                          void* stream) {
  if (nq <= 0) return 0;
  if (L < 1 || L > 64) return -1;
  const int lcap = std::max(1, kout);  // a merged list holds up to k <= kout entries
  const size_t lds = 2 * (size_t)L * lcap * (sizeof(double) + sizeof(int));
  if (L <= 8) {  // one lane per query, heads in registers (writes every slot of [0, kout))
    const dim3 g((nq + 255) / 256), b(256);
    hipStream_t st = (hipStream_t)stream;
    // 16-byte window loads: every list start (l * list_stride + q * kin) must be 4-aligned too
    const bool win = kin % 4 == 0 && list_stride % 4 == 0 && ((uintptr_t)in_d & 15) == 0 &&
                     ((uintptr_t)in_i & 15) == 0 &&
                     !(getenv("DMLP_MERGE_WIN") && getenv("DMLP_MERGE_WIN")[0] == '0');
    if (win) {
#define DMLP_MERGE_WIN(LV)                                                                     \
  case LV:                                                                                     \
    hipLaunchKernelGGL(k_merge_win<LV>, g, b, 0, st, in_d, in_i, list_stride, kin, qk, nq, out_d, \
                       out_i, kout);                                                           \
    break;
      switch (L) {
        DMLP_MERGE_WIN(1) DMLP_MERGE_WIN(2) DMLP_MERGE_WIN(3) DMLP_MERGE_WIN(4)
        DMLP_MERGE_WIN(5) DMLP_MERGE_WIN(6) DMLP_MERGE_WIN(7) DMLP_MERGE_WIN(8)
      }
#undef DMLP_MERGE_WIN
      DMLP_LAUNCH_CHECK();
      return 0;
    }
#define DMLP_MERGE_SEQ(LV)                                                                     \
  case LV:                                                                                     \
    hipLaunchKernelGGL(k_merge_seq<LV>, g, b, 0, st, in_d, in_i, list_stride, kin, qk, nq, out_d, \
                       out_i, kout);                                                           \
    break;
    switch (L) {
      DMLP_MERGE_SEQ(1) DMLP_MERGE_SEQ(2) DMLP_MERGE_SEQ(3) DMLP_MERGE_SEQ(4)
      DMLP_MERGE_SEQ(5) DMLP_MERGE_SEQ(6) DMLP_MERGE_SEQ(7) DMLP_MERGE_SEQ(8)
    }
#undef DMLP_MERGE_SEQ
  } else if (lds <= 48 * 1024) {  // LDS-resident merge path (P <= 8 lists of k <= 256, ...)
    const int w = lds <= 12 * 1024 ? 4 : 1;  // queries (waves) per workgroup
    hipLaunchKernelGGL(k_merge_path, dim3((nq + w - 1) / w), dim3(64 * w), lds * w,
                       (hipStream_t)stream, in_d, in_i, L, list_stride, kin, qk, nq, out_d, out_i,
                       kout, lcap);
  } else {
    hipLaunchKernelGGL(k_merge, dim3((nq + 3) / 4), dim3(256), 0, (hipStream_t)stream, in_d,
                       in_i, L, list_stride, kin, qk, nq, out_d, out_i, kout);
  }
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_finalize(const double* d, const int* ids, int kstride, const int* qk,
                             const int* qidx, int nq, const int* labels, int label_lo, int label_hi, int* out_label,
                             uint64_t* out_cs, void* stream) {
  if (nq <= 0) return 0;
  hipLaunchKernelGGL(k_finalize, dim3((nq + 3) / 4), dim3(256), 0, (hipStream_t)stream, d, ids,
                     kstride, qk, qidx, nq, labels, label_lo, label_hi, out_label, out_cs);
  DMLP_LAUNCH_CHECK();
  return 0;
}

namespace {
__global__ void k_fill_f64(double* __restrict__ p, int64_t n, double v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
}  // namespace

namespace {
__global__ void k_offset_ids(int* __restrict__ ids, int64_t n, int off) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (ids[i] >= 0) ids[i] += off;
}
}  // namespace

// shard-local ids -> global ids (padding -1 kept)
extern "C" int dmlp_offset_ids(int* ids, int64_t n, int off, void* stream) {
  if (n <= 0 || off == 0) return 0;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_offset_ids, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, ids,
                     n, off);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_fill_f64(double* p, int64_t n, double v, void* stream) {
  if (n <= 0) return 0;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_fill_f64, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p, n,
                     v);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int64_t dmlp_format_bound(int nq) { return (int64_t)nq * 48 + 64; }

// lines per format block: 256 (512 blocks for the headline's 131072 lines push the report's
// PCIe writes from more CUs than 1024-line blocks: 106.5 vs 109.4 us, profiles/r12k_fmt_block_ab.txt)
constexpr int kFmtBlock = 256;

// line_off needs nq + 1 + (nq/FB + 2) int64 of scratch; on completion line_off[nq] = bytes.
extern "C" int64_t dmlp_format_scratch(int nq) {
  return (int64_t)nq + 1 + (nq + kFmtBlock - 1) / kFmtBlock + 1;
}

extern "C" int dmlp_format_report(const uint64_t* cs, int nq, int qid_base, int64_t* line_off,
                                  char* out, void* stream) {
  return dmlp_format_report_at(cs, nq, qid_base, line_off, out, nullptr, stream);
}

// The same, the lines starting at byte *base of out (device word; null: 0): a report rendered in
// query parts, each part's base = the previous part's line_off[nq] (its absolute end)
extern "C" int dmlp_format_report_at(const uint64_t* cs, int nq, int qid_base, int64_t* line_off,
                                     char* out, const int64_t* base, void* stream) {
  if (nq <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (nq + kFmtBlock - 1) / kFmtBlock;
  int64_t* blocksum = line_off + nq + 1;
  hipLaunchKernelGGL(k_fmt_len<kFmtBlock>, dim3(nb), dim3(kFmtBlock), 0, st, cs, nq, qid_base,
                     line_off, blocksum);
  DMLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_fmt_scan_blocks, dim3(1), dim3(1024), 0, st, blocksum, nb);
  DMLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_fmt_write<kFmtBlock>, dim3(nb), dim3(kFmtBlock), 0, st, cs, nq, qid_base,
                     line_off, blocksum, base, out);
  DMLP_LAUNCH_CHECK();
  return 0;
}
