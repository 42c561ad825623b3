// screen_stream.hip — barrier-free streaming variant of the bf16x3 MFMA screen (numerics as in
// screen.hip: score a = <q',x'> - |x'|^2/2 in fp32 from a 3-term bf16 split, per-query
// threshold h = a_k - 2*eps_q that only rises, exact fp64 re-rank in refine.hip).
//
// Why a second kernel: profiling the LDS-shared kernel (profiles/README.md) showed its per-tile
// workgroup barrier coupling 8 waves, so one wave's candidate appends / threshold compactions
// stalled the other seven.  Here every wave is its own workgroup and nothing couples waves:
//   * a wave owns 16*CT queries (CT MFMA column tiles, 64 at CT = 4) for its data slice, so
//     every A fragment it fetches feeds CT x 3 MFMAs;
//   * the slice streams in 16-point steps (one MFMA row tile): the step's fragments come
//     straight from L2 / Infinity Cache into a D-deep register ring (global_load_dwordx4 issued
//     D steps ahead) — no LDS staging, no barrier;
//   * acc is double-buffered: the MFMAs of step j are issued before the candidate epilogue of
//     step j-1 runs, so the VALU work overlaps the matrix pipe;
//   * a lane appends at most 4 entries per column per step into its own LDS sub-buffer
//     (4 per column, SUB entries each), so appends need no cross-lane coordination; as soon as
//     a sub-buffer passes SUB-4 entries, the column's threshold is tightened (20-round ballot
//     radix select of the k-th score) and survivors are re-dealt round-robin.  Column state
//     (h, k, eps, counts) lives in LDS so the compaction code exists once, not per column tile.
// Registers stay under 256 VGPRs (no AGPR copies); LDS = 36.6 KiB, four waves (one per SIMD)
// per CU.
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

namespace {

int g_stream_mode = 0;  // profiling ablations (bit 0 no candidates, 1 no MFMA, 2 no streaming,
                        // 3 event counters into g_stream_dbg, 4 s_memtime cycle accounting)
int g_stream_groups = 1;  // 1: append 4-row groups (one entry per column tile and step)
__device__ unsigned long long g_stream_dbg[8];

// Wave-wide max / min of a u32 through DPP row shifts + row broadcasts (no LDS traffic; the
// __shfl_xor form lowers to six dependent ds_bpermute round trips).  Result is wave-uniform.
template <bool MAX>
__device__ __forceinline__ unsigned wave_reduce_u32(unsigned v) {
  const int idn = MAX ? 0 : -1;
#define DMLP_DPP_STEP(CTRL, ROWMASK)                                                          \
  {                                                                                           \
    const unsigned o_ = (unsigned)__builtin_amdgcn_update_dpp(idn, (int)v, CTRL, ROWMASK, 0xf, false); \
    v = MAX ? (v > o_ ? v : o_) : (v < o_ ? v : o_);                                          \
  }
  DMLP_DPP_STEP(0x111, 0xf)  // row_shr:1
  DMLP_DPP_STEP(0x112, 0xf)  // row_shr:2
  DMLP_DPP_STEP(0x114, 0xf)  // row_shr:4
  DMLP_DPP_STEP(0x118, 0xf)  // row_shr:8  -> lane 15 of each row holds the row's result
  DMLP_DPP_STEP(0x142, 0xa)  // row_bcast:15 into rows 1, 3
  DMLP_DPP_STEP(0x143, 0xc)  // row_bcast:31 into rows 2, 3 -> lane 63 holds the wave's
#undef DMLP_DPP_STEP
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

template <int KT, int CT, int SUB, bool G>
struct StreamCfg {
  static constexpr int CAP = 4 * SUB;             // buffered entries per (query, slice)
  static constexpr int APPEND = G ? 1 : 4;        // entries a lane appends per column and step
  static constexpr int IDCAP = G ? 4 * CAP : CAP; // candidate ids written per (query, slice)
  static constexpr int QW = 16 * CT;              // queries per wave / workgroup
  static constexpr int NCOL = QW;
  static constexpr int FRAGS = 4 * KT * 2;        // 1 KiB fragments per 64-point tile
  static constexpr int SUB_BYTES = NCOL * 4 * (SUB + 1) * 8;
  static constexpr int LDS = SUB_BYTES + NCOL * 4 * 4 + NCOL * 4 * 3;
  static constexpr int D = 4;                     // register-ring depth (steps in flight)
  static_assert(CAP <= 64, "one buffered entry per lane in compaction");
};

template <int KT, int CT, int SUB, int mode, bool G>
__global__ __launch_bounds__(64) void k_screen_stream(
    const u32x4* __restrict__ xfrag, const f32x4* __restrict__ xinit4, int n_tiles,
    const bf16x8* __restrict__ qhi, const bf16x8* __restrict__ qlo, const float* __restrict__ qn,
    const int* __restrict__ qidx, const int* __restrict__ qk, int nq,
    const unsigned* __restrict__ xnmax_bits, const unsigned* __restrict__ bad, float eps_rel,
    int S, int tiles_per_slice, int n_qblocks, int* __restrict__ cand_ids,
    int* __restrict__ cand_cnt) {
  using C = StreamCfg<KT, CT, SUB, G>;
  constexpr int CAP = C::CAP;
  constexpr int APPEND = C::APPEND;
  constexpr int D = C::D;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  i32x2* const sbuf = (i32x2*)smem;                               // sub-buffers
  int* const lcnt = (int*)(smem + C::SUB_BYTES);                   // [col][m] counts
  float* const lh = (float*)(lcnt + C::NCOL * 4);                  // [col] threshold
  int* const lk = (int*)(lh + C::NCOL);                            // [col] k
  float* const leps = (float*)(lk + C::NCOL);                      // [col] eps

  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int kg = lane >> 4;

  // ---- block -> (query block, slice); XCD-aware when S % 8 == 0 (see screen.hip)
  const int b = blockIdx.x;
  int qb, s;
  if ((S & 7) == 0) {
    const int xcd = b & 7, local = b >> 3, m = S >> 3;
    const int sl = local / n_qblocks;
    qb = local - sl * n_qblocks;
    s = xcd * m + sl;
  } else {
    s = b % S;
    qb = b / S;
  }
  const int t0 = s * tiles_per_slice;
  int t1 = t0 + tiles_per_slice;
  if (t1 > n_tiles) t1 = n_tiles;
  const int nt = t1 > t0 ? t1 - t0 : 0;
  const int nsteps = nt * 4;
  const int pbase = qb * C::QW;

  if (*bad) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int p = pbase + ct * 16 + c;
      if (lane < 16 && p < nq) cand_cnt[(int64_t)p * S + s] = -1;
    }
    return;
  }
  const float xnmax = __uint_as_float(*xnmax_bits);

  // ---- per column tile: query fragments, threshold (register copy), own sub-buffer count
  bf16x8 bh[CT][KT], bl[CT][KT];
  float h[CT];
  int cnt[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int p = pbase + ct * 16 + c;
    const bool valid = p < nq;
    const int q = valid ? qidx[p] : 0;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      bh[ct][kt] = qhi[(q * KT + kt) * 4 + kg];
      bl[ct][kt] = qlo[(q * KT + kt) * 4 + kg];
    }
    h[ct] = valid ? -FLT_MAX : INFINITY;
    cnt[ct] = 0;
    if (lane < 16) {
      const int col = ct * 16 + c;
      lh[col] = h[ct];
      lk[col] = valid ? qk[q] : 0;
      leps[col] = eps_rel * (qn[q] + xnmax);
    }
  }
  // sub-buffer (col, m): pitch SUB+1 keeps a lane group's 16 columns on distinct banks
  auto sub_ptr = [&](int col, int m) {
    return sbuf + (((col >> 4) * 4 + m) * 16 + (col & 15)) * (SUB + 1);
  };

  // (mode & 16) cycle accounting: loop, compaction, append path (s_memtime, core clock)
  unsigned long long t_comp = 0, t_app = 0;

  // ---- compaction of every column whose sub-buffer passed SUB-4 (state in LDS, runtime loop)
  auto compact_pending = [&]() {
    const unsigned long long tc0_ = (mode & 16) ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) lcnt[(ct * 16 + c) * 4 + kg] = cnt[ct];
    dmlp::wave_sync();
    unsigned long long pend = 0;  // bit col
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const unsigned long long bm = __ballot(cnt[ct] > SUB - APPEND);
      pend |= ((bm | (bm >> 16) | (bm >> 32) | (bm >> 48)) & 0xffffull) << (16 * ct);
    }
    if ((mode & 8) && lane == 0) atomicAdd(&g_stream_dbg[3], (unsigned long long)__popcll(pend));
    while (pend) {
      const int col = __ffsll((long long)pend) - 1;
      pend &= pend - 1;
      // all of the column's state in one batch of LDS reads (one latency, not five)
      const int nmine = lcnt[col * 4 + kg];
      const i32x2 eraw = sub_ptr(col, kg)[c];  // slot c < SUB+1 always exists
      const int kc = __builtin_amdgcn_readfirstlane(lk[col]);
      float hc = lh[col];
      const float epc = leps[col];
      const bool ok = c < nmine;
      const i32x2 e = ok ? eraw : (i32x2){__float_as_int(-INFINITY), -1};
      const int ntot = __popcll(__ballot(ok));
      if (ntot >= kc) {
        const unsigned bits = (unsigned)e.x;
        const unsigned u = ok ? (bits ^ ((bits >> 31) ? 0xffffffffu : 0x80000000u)) : 0u;
        // the k-th largest key lies in [min, max] of the buffered keys: the radix search
        // starts below their common prefix (DPP reductions, no LDS round trips), and runs as
        // a scalar loop (T, bit uniform in SGPRs)
        const unsigned umx = wave_reduce_u32<true>(u);
        const unsigned umn = wave_reduce_u32<false>(ok ? u : 0xffffffffu);
        const unsigned dif = umx ^ umn;
        const int top = dif ? 31 - __clz((int)dif) : -1;
        unsigned T = umx;  // top < 0: every buffered key is equal
        if (top >= 31) T = 0u;
        else if (top >= 0) T = umx & ~((2u << top) - 1u);
#pragma unroll 1
        for (int bit = top; bit >= 12; --bit) {  // low bits left 0: T <= exact k-th key
          const unsigned cand = T | (1u << bit);
          if (__popcll(__ballot(u >= cand)) >= kc) T = cand;
        }
        const float ak = __uint_as_float((T >> 31) ? (T ^ 0x80000000u) : ~T);
        hc = fmaxf(hc, ak - 2.0f * epc);
      }
      const bool keep = ok && __int_as_float(e.x) >= hc;
      const unsigned long long km = __ballot(keep);
      const int kept = __popcll(km);
      dmlp::wave_sync();
      if (keep) {
        const int pos = __popcll(km & dmlp::lanemask_lt());
        sub_ptr(col, pos & 3)[pos >> 2] = e;
      }
      if (lane < 4)
        lcnt[col * 4 + lane] = kept > 4 * (SUB - APPEND) ? -(1 << 28) : (kept + 3 - lane) >> 2;
      if (lane == 0) lh[col] = kept > 4 * (SUB - APPEND) ? INFINITY : hc;  // overflow: exact path
      dmlp::wave_sync();
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      cnt[ct] = lcnt[(ct * 16 + c) * 4 + kg];
      h[ct] = lh[ct * 16 + c];
    }
    // resolve these LDS loads here: otherwise the waitcnt pass sees h / cnt possibly pending
    // at the merge after `if (trig) compact_pending()` and makes EVERY following step wait
    // for all outstanding LDS traffic (i.e. the previous step's appends)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if (mode & 16) t_comp += __builtin_amdgcn_s_memtime() - tc0_;
  };

  // ---- D-deep register ring of step fragments + double-buffered accumulators
  bf16x8 A[D][KT][2];
  f32x4 Xi[D];
  f32x4 acc[2][CT];
  // step j covers tile t0 + j/4, row tile j%4; within the unrolled body j%4 == r is static
#define DMLP_LOAD(J, R)                                                                         \
  do {                                                                                          \
    const int jj_ = (J) < nsteps ? (J) : nsteps - 1;                                            \
    const int t_ = t0 + (jj_ >> 2);                                                             \
    const int rt_ = jj_ & 3;                                                                    \
    const u32x4* src_ = xfrag + (int64_t)t_ * (C::FRAGS * 64) + lane;                          \
    _Pragma("unroll") for (int kt = 0; kt < KT; ++kt) {                                         \
      A[R][kt][0] = __builtin_bit_cast(bf16x8, src_[((rt_ * KT + kt) * 2 + 0) * 64]);           \
      A[R][kt][1] = __builtin_bit_cast(bf16x8, src_[((rt_ * KT + kt) * 2 + 1) * 64]);           \
    }                                                                                           \
    Xi[R] = xinit4[(int64_t)t_ * 16 + rt_ * 4 + kg];                                            \
  } while (0)
#define DMLP_MFMA(R, AB)                                                                        \
  do {                                                                                          \
    if (!(mode & 2)) {                                                                          \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                       \
        acc[AB][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][0][0], bh[ct][0], Xi[R], 0, 0, 0); \
        acc[AB][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][0][0], bl[ct][0], acc[AB][ct], 0, 0, 0); \
        acc[AB][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][0][1], bh[ct][0], acc[AB][ct], 0, 0, 0); \
        _Pragma("unroll") for (int kt = 1; kt < KT; ++kt) {                                     \
          acc[AB][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][kt][0], bh[ct][kt], acc[AB][ct], 0, 0, 0); \
          acc[AB][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][kt][0], bl[ct][kt], acc[AB][ct], 0, 0, 0); \
          acc[AB][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][kt][1], bh[ct][kt], acc[AB][ct], 0, 0, 0); \
        }                                                                                       \
      }                                                                                         \
    } else {                                                                                    \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) acc[AB][ct] = Xi[R];                    \
    }                                                                                           \
  } while (0)
#define DMLP_EPILOGUE(AB, J)                                                                    \
  do {                                                                                          \
    const int jj_ = (J);                                                                        \
    const int idbase_ = (t0 + (jj_ >> 2)) * 64 + (jj_ & 3) * 16 + kg * 4;                       \
    float m_[CT];                                                                               \
    bool any_ = false;                                                                          \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                         \
      m_[ct] = fmaxf(fmaxf(acc[AB][ct][0], acc[AB][ct][1]), fmaxf(acc[AB][ct][2], acc[AB][ct][3])); \
      any_ |= m_[ct] >= h[ct];                                                                  \
    }                                                                                           \
    if ((mode & 8) && lane == 0) atomicAdd(&g_stream_dbg[0], 1ull);                             \
    if ((mode & 1) == 0 && __ballot(any_)) {                                                    \
      if (mode & 8) {                                                                           \
        int np_ = 0;                                                                            \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct)                                       \
          _Pragma("unroll") for (int j = 0; j < 4; ++j) np_ += acc[AB][ct][j] >= h[ct];         \
        for (int o_ = 32; o_ > 0; o_ >>= 1) np_ += __shfl_xor(np_, o_);                         \
        if (lane == 0) { atomicAdd(&g_stream_dbg[1], 1ull);                                     \
                         atomicAdd(&g_stream_dbg[2], (unsigned long long)np_); }                \
      }                                                                                         \
      /* branch-free appends: every lane writes each value to its next free slot and only  \
         advances the slot on a hit (slots cnt..cnt+3 <= SUB-1 exist; a miss is overwritten  \
         later and never read).  Per-lane branches here cost a taken s_cbranch each. */      \
      const unsigned long long ta0_ = (mode & 16) ? __builtin_amdgcn_s_memtime() : 0;         \
      bool trig_ = false;                                                                       \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                       \
        i32x2* mys_ = sub_ptr(ct * 16 + c, kg);                                                 \
        int cn_ = cnt[ct];                                                                      \
        if (G) {                                                                                \
          /* one entry per lane, column and step: the 4-row group (ids idbase..idbase+3)     \
             scored by its max; the k-th largest group max is still a lower bound on a_k */   \
          const int mk_ = (acc[AB][ct][0] >= h[ct] ? 1 : 0) | (acc[AB][ct][1] >= h[ct] ? 2 : 0) | \
                          (acc[AB][ct][2] >= h[ct] ? 4 : 0) | (acc[AB][ct][3] >= h[ct] ? 8 : 0);  \
          /* (group base << 2) | member hit mask: members below the threshold at append time  \
             can never re-enter (h only rises), so the final write emits only masked ids */   \
          mys_[cn_] = (i32x2){__float_as_int(m_[ct]), ((idbase_ - t0 * 64) << 2) | mk_};        \
          cn_ += m_[ct] >= h[ct] ? 1 : 0;                                                       \
        } else {                                                                                \
          _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                       \
            mys_[cn_] = (i32x2){__float_as_int(acc[AB][ct][j]), idbase_ + j};                   \
            cn_ += acc[AB][ct][j] >= h[ct] ? 1 : 0;                                             \
          }                                                                                     \
        }                                                                                       \
        cnt[ct] = cn_;                                                                          \
        trig_ |= cn_ > SUB - APPEND;                                                            \
      }                                                                                         \
      if (mode & 16) {                                                                          \
        __builtin_amdgcn_s_waitcnt(0xC07F);                                                     \
        t_app += __builtin_amdgcn_s_memtime() - ta0_;                                           \
      }                                                                                         \
      if (__ballot(trig_)) compact_pending();                                                   \
    }                                                                                           \
  } while (0)

  const unsigned long long tl0_ = (mode & 16) ? __builtin_amdgcn_s_memtime() : 0;
  if (nsteps > 0) {
#pragma unroll
    for (int r = 0; r < D; ++r) DMLP_LOAD(r, r);
    for (int j0 = 0; j0 < nsteps; j0 += D) {
#pragma unroll
      for (int r = 0; r < D; ++r) {
        const int j = j0 + r;  // nsteps % 4 == 0 and D == 4: j < nsteps inside the body
        DMLP_MFMA(r, r & 1);
        if (!(mode & 4)) DMLP_LOAD(j + D, r);
        if (j > 0) DMLP_EPILOGUE((r + 1) & 1, j - 1);
      }
    }
    DMLP_EPILOGUE((nsteps - 1) & 1, nsteps - 1);
  }
  if ((mode & 16) && lane == 0) {
    atomicAdd(&g_stream_dbg[4], __builtin_amdgcn_s_memtime() - tl0_);
    atomicAdd(&g_stream_dbg[5], t_comp);
    atomicAdd(&g_stream_dbg[6], t_app);
  }
  if (mode & 1) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) asm volatile("" ::"v"(acc[0][ct]), "v"(acc[1][ct]));
  }
#undef DMLP_LOAD
#undef DMLP_MFMA
#undef DMLP_EPILOGUE

  // ---- write this slice's candidates (ids only; refine recomputes exact distances)
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) lcnt[(ct * 16 + c) * 4 + kg] = cnt[ct];
  dmlp::wave_sync();
  for (int col = 0; col < C::NCOL; ++col) {
    const int pp = pbase + col;
    if (pp >= nq) break;
    int* out = cand_ids + ((int64_t)pp * S + s) * C::IDCAP;
    if (lcnt[col * 4] < 0) {
      if (lane == 0) cand_cnt[(int64_t)pp * S + s] = -1;
      continue;
    }
    const int nmine = lcnt[col * 4 + kg];
    const bool ok = c < nmine;
    const i32x2 e = ok ? sub_ptr(col, kg)[c] : (i32x2){0, -1};
    const float hc = lh[col];
    const bool keep = ok && __int_as_float(e.x) >= hc;
    if (G) {
      // expand kept groups to the members that were above the threshold when appended
      // (padding members score -inf and are never in the mask)
      const int gbase = ((e.y >> 2) & ~3) + t0 * 64;  // slice-relative group base
      int nout = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool v = keep && ((e.y >> j) & 1);
        const unsigned long long mj = __ballot(v);
        if (v) out[nout + __popcll(mj & dmlp::lanemask_lt())] = gbase + j;
        nout += __popcll(mj);
      }
      if (lane == 0) cand_cnt[(int64_t)pp * S + s] = nout;
    } else {
      const unsigned long long m = __ballot(keep);
      if (keep) out[__popcll(m & dmlp::lanemask_lt())] = e.y;
      if (lane == 0) cand_cnt[(int64_t)pp * S + s] = __popcll(m);
    }
  }
}

template <int KT, int CT, int SUB, bool G>
int launch_stream(const void* xfrag, const float* xinit, int64_t n_tiles, const void* qhi,
                  const void* qlo, const float* qn, const int* qidx, const int* qk, int nq,
                  const unsigned* xnmax, const unsigned* bad, float eps_rel, int S,
                  int* cand_ids, int* cand_cnt, hipStream_t stream) {
  using C = StreamCfg<KT, CT, SUB, G>;
  const int n_qblocks = (nq + C::QW - 1) / C::QW;
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S;
  if (grid <= 0) return 0;
  // the ablation mode is a template parameter: a runtime branch in the hot loop made hipcc
  // hoist the ablation's register copies and drain vmcnt every iteration
#define DMLP_STREAM_LAUNCH(M)                                                                  \
  hipLaunchKernelGGL((k_screen_stream<KT, CT, SUB, M, G>), dim3((unsigned)grid), dim3(64), C::LDS, \
                     stream, (const u32x4*)xfrag, (const f32x4*)xinit, (int)n_tiles,           \
                     (const bf16x8*)qhi, (const bf16x8*)qlo, qn, qidx, qk, nq, xnmax, bad,     \
                     eps_rel, S, tps, n_qblocks, cand_ids, cand_cnt)
  switch (g_stream_mode) {
    case 1: DMLP_STREAM_LAUNCH(1); break;
    case 3: DMLP_STREAM_LAUNCH(3); break;
    case 5: DMLP_STREAM_LAUNCH(5); break;
    case 7: DMLP_STREAM_LAUNCH(7); break;
    case 8: DMLP_STREAM_LAUNCH(8); break;
    case 16: DMLP_STREAM_LAUNCH(16); break;
    default: DMLP_STREAM_LAUNCH(0); break;
  }
#undef DMLP_STREAM_LAUNCH
  DMLP_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// Streaming screen for k <= 32 and A <= 64 (KT <= 2); 64 queries per workgroup.  Candidate
// ids per (query, slice): dmlp_screen_stream_cap(kmax) for the class's largest k.  Group mode
// with kmax <= 16 uses 8-entry sub-buffers (19.8 KiB LDS: two waves per SIMD, so one wave's
// candidate work overlaps the other's MFMAs); otherwise 16 (36.6 KiB, one wave per SIMD).
int g_stream_sub = 0;  // 0 auto, 8 / 16 forced (A/B)
static int stream_sub(int kmax) {
  if (g_stream_sub) return g_stream_sub;
  return (g_stream_groups && kmax <= 16) ? 8 : 16;
}
extern "C" int dmlp_screen_stream_qw(int KT) { return (KT == 1 || KT == 2) ? 64 : 0; }
extern "C" int dmlp_screen_stream_cap(int kmax) {
  return 4 * stream_sub(kmax) * (g_stream_groups ? 4 : 1);
}
extern "C" int dmlp_screen_stream_kmax(void) { return 32; }
// resident workgroups (= waves) per CU of the variant chosen for kmax (LDS-bound)
extern "C" int dmlp_screen_stream_waves_per_cu(int kmax) { return stream_sub(kmax) == 8 ? 8 : 4; }
extern "C" void dmlp_set_stream_sub(int sub) { g_stream_sub = (sub == 8 || sub == 16) ? sub : 0; }

extern "C" void dmlp_set_stream_mode(int mode) { g_stream_mode = mode; }
extern "C" void dmlp_set_stream_groups(int on) { g_stream_groups = on ? 1 : 0; }

extern "C" int dmlp_stream_debug_counters(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stream_dbg), sizeof(g_stream_dbg));
  if (e != hipSuccess) return -(int)e;
  if (reset) {
    unsigned long long z[8] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_stream_dbg), z, sizeof(z));
    if (e != hipSuccess) return -(int)e;
  }
  return 0;
}

extern "C" int dmlp_screen_stream(int KT, const void* xfrag, const float* xinit, int64_t n_tiles,
                                  const void* qhi, const void* qlo, const float* qn,
                                  const int* qidx, const int* qk, int nq, int kmax,
                                  const unsigned* xnmax_bits, const unsigned* bad, float eps_rel,
                                  int S, int* cand_ids, int* cand_cnt, void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || n_tiles < 0 || n_tiles > 0x7fffffff / 64) return -1;
  // group entries carry slice-relative ids << 2: a slice must stay below 2^29 points
  if ((n_tiles + S - 1) / S > (1 << 29) / 64) return -4;
  if (kmax > 32) return -3;
  hipStream_t st = (hipStream_t)stream;
  const int sub = stream_sub(kmax);
  if (sub == 8 && kmax > 16) return -3;
#define DMLP_STREAM_ARGS xfrag, xinit, n_tiles, qhi, qlo, qn, qidx, qk, nq, xnmax_bits, bad, \
                         eps_rel, S, cand_ids, cand_cnt, st
#define DMLP_STREAM_KT(KTV)                                                                    \
  if (g_stream_groups)                                                                         \
    return sub == 8 ? launch_stream<KTV, 4, 8, true>(DMLP_STREAM_ARGS)                         \
                    : launch_stream<KTV, 4, 16, true>(DMLP_STREAM_ARGS);                       \
  return launch_stream<KTV, 4, 16, false>(DMLP_STREAM_ARGS);
  if (KT == 1) { DMLP_STREAM_KT(1) }
  if (KT == 2) { DMLP_STREAM_KT(2) }
#undef DMLP_STREAM_KT
#undef DMLP_STREAM_ARGS
  return -2;
}
