// screen_x2.hip — single-term bf16 screen on v_mfma_f32_32x32x16_bf16 (K2 + K3 screen half).
//
// Same output contract as screen_x1.hip (4-point group entries per (query, slice) + the slice
// threshold / error bound in cand_h, consumed unchanged by refine.hip's group refine), a
// different balance of the CDNA4 pipes:
//
//  * Shape.  A workgroup is 8 waves (2 per SIMD) x T = 2 query tiles of 32 queries = 512
//    queries, streaming the data in 32-point steps.  Per step and tile, 2*KT MFMAs of 32x32x16
//    give the 32 x 32 scores.  A 32x32 MFMA holds vector issue for 8 of its 32 cycles
//    (16x16x32: 8 of 16) and the SIMD's other wave issues its epilogue meanwhile, so the
//    epilogue has ~3x the VALU slots per score of screen_x1.
//  * Data through LDS.  The 8 waves share every step's A operand (2 KiB hi image per KT) and
//    its xinit row terms through an 8-step LDS ring: each wave register-stages 1/8 of a 2-step
//    phase (global -> VGPR two phases ahead, -> LDS two phases ahead of use), one s_barrier per
//    phase.  L2 traffic is 1/8 of a per-wave stream (that form measured L2-bound at ~12 TB/s).
//  * C operand.  The -|x'|^2/2 row terms are staged into the ring permuted to the 32x32 C/D
//    layout ([half][register]), so a lane's 16 C values are one 64-byte LDS read (a broadcast:
//    32 lanes read each address), shared by the T tiles of the step; no VALU.
//  * Epilogue.  Lane l of a tile holds query column l & 31 and rows (r & 3) + 8 (r >> 2) +
//    4 (l >> 5), i.e. 4 runs u of 4 consecutive points.  Run maxima (v_max3), the tile max and
//    one compare are the fast path; a wave-uniform branch per tile (any lane at or above its
//    threshold) guards exec-masked appends per run.  Run u of half hh in step j is the 4-point
//    group g = 8 j + 2 u + hh (points 4g .. 4g+3 of the slice): screen_x1's group numbering.
//  * Candidate buffers.  4-byte entries (top 16 bits of the fp32 run max | 16-bit group index),
//    one sub-buffer of SUB slots per (lane, tile): a column's entries live in lanes c and c+32.
//    A sub-buffer saturates into a pad slot (a full one counts as overflow, never a stray
//    write).  When any sub-buffer of a wave passes its limit, that wave compacts its 64 columns
//    at once (lane j owns column (j >> 5, j & 31); its threshold state lives in its registers):
//    radix select of the k-th largest key over <= 2 SUB entries, h = key_k - 2 eps (a lower
//    bound on a_k - eps), survivors re-dealt in place over the column's two sub-buffers.
//
// Error bound: screen_x1.hip's (dmlp_screen_x1_bound) — the same single-term products and the
// same fp32 C term, summed in a different order (the bound holds for any order).
// Reference: the distance / top-k hot loop of engine.cpp:233-257, bench_4 @0xcb80 (SURVEY §2.5
// K2/K3); group refine and exactness: refine.hip.
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

#include <type_traits>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

int g_x2_mode = 0;  // profiling: 1 = no candidate path (pure MFMA + max loop), 8 = counters
// MODE 8 event counters (summed over waves): tile branches taken, entries appended, compactions,
// cycles in compactions, cycles waiting at the phase barrier, cycles in the main loop
__device__ unsigned long long g_x2_dbg[8];

__device__ __forceinline__ unsigned ord32(unsigned b) {
  return b ^ ((unsigned)((int)b >> 31) | 0x80000000u);
}
__device__ __forceinline__ unsigned unord32(unsigned o) {
  return o ^ ((o >> 31) ? 0x80000000u : 0xffffffffu);
}

constexpr int kX2IdCap = 46;  // candidate id stride per (query, slice): the largest CAPE

template <int KT, int SUB, bool PW = false>
struct X2Cfg {
  static constexpr int T = 2;               // query tiles per wave
  static constexpr int W = PW ? 1 : 8;      // waves per workgroup (PW: per-wave streaming)
  static constexpr int NCOL = 32 * T;       // queries per wave
  static constexpr int NQ = W * NCOL;       // queries per workgroup
  static constexpr int KS = 2 * KT;         // 16-deep k-steps per 32-point step
  static constexpr int CP = SUB + 1;        // words per (lane, tile) sub-buffer: SUB slots + pad
  // compactions run at phase starts, after a wave flagged a sub-buffer past LIMN in the
  // previous phase; a lane appends at most one entry per run (4) per step, two steps per phase
  static constexpr int LIMN = SUB - 9;
  static constexpr int CAPE = 2 * LIMN;     // group entries a column may keep
  static constexpr int STEPB = 2 * KT * 1024;             // hi image bytes per 32-point step
  static constexpr int RING = 8;                          // steps in the LDS ring (4 phases)
  static constexpr int SB_WAVE = T * 64 * CP * 4;         // candidate sub-buffers per wave
  static constexpr int OFF_X = W * SB_WAVE;               // xinit ring [RING][32] fp32
  static constexpr int OFF_A = OFF_X + RING * 128;        // A ring [RING][STEPB]
  static constexpr int OFF_F = OFF_A + RING * STEPB;       // compaction-event flags [3]
  // per-wave form: + a C-operand ring of two 4-step windows (4 x 32 rows of -|x'|^2/2 each),
  // stored in the C/D register layout so a lane's 16 C values are one 64-byte broadcast read
  static constexpr int XRW = 2 * 4 * 128;
  static constexpr int LDS = PW ? SB_WAVE + XRW : OFF_F + 16;
  static constexpr int LDB = 8 * KT;                      // staged bytes per lane and phase
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(CAPE <= kX2IdCap, "id stride");
};

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) unsigned lds_u32;

// raw buffer descriptor (stride 0, num_records bytes, range-checked: out-of-range loads read 0)
__device__ __forceinline__ i32x4 buffer_desc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 d;
  d.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  d.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xffff);
  d.z = __builtin_amdgcn_readfirstlane(bytes);
  d.w = 0x00020000;
  return d;
}

template <int I>
__device__ __forceinline__ float row_bcast(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + I,
                                                            0xf, 0xf, false));
}

// C block from one value per lane: register i = lane (16 g + i)'s value, broadcast within each
// 16-lane row (v_mov_b32_dpp row_newbcast)
__device__ __forceinline__ f32x16 c_block(float v) {
  f32x16 r;
  r[0] = row_bcast<0>(v); r[1] = row_bcast<1>(v); r[2] = row_bcast<2>(v); r[3] = row_bcast<3>(v);
  r[4] = row_bcast<4>(v); r[5] = row_bcast<5>(v); r[6] = row_bcast<6>(v); r[7] = row_bcast<7>(v);
  r[8] = row_bcast<8>(v); r[9] = row_bcast<9>(v); r[10] = row_bcast<10>(v);
  r[11] = row_bcast<11>(v); r[12] = row_bcast<12>(v); r[13] = row_bcast<13>(v);
  r[14] = row_bcast<14>(v); r[15] = row_bcast<15>(v);
  return r;
}

template <int KT>
struct Stage {  // one phase's register-staged share of a wave
  typedef typename std::conditional<KT == 1, u32x2, u32x4>::type A;
  A a;
  float x;
};

template <int KT, int SUB, int MODE, bool PW>
__global__ __launch_bounds__(PW ? 64 : 512) __attribute__((amdgpu_waves_per_eu(2))) void k_screen_x2(
    const u32x4* __restrict__ xfrag, const float* __restrict__ xinit, int n_tiles,
    const bf16x8* __restrict__ qhi, const float* __restrict__ qn, const int* __restrict__ qidx,
    const int* __restrict__ qk, int nq, const unsigned* __restrict__ xnmax_bits,
    const unsigned* __restrict__ bad, float r1, float r2, int S, int tiles_per_slice,
    int n_qblocks, int hl, int* __restrict__ cand_ids, int* __restrict__ cand_cnt,
    float* __restrict__ cand_h) {
  using C = X2Cfg<KT, SUB, PW>;
  constexpr int T = C::T;
  constexpr int KS = C::KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int c = lane & 31;
  const int hh = lane >> 5;
  unsigned* const sbuf = (unsigned*)(smem + w * C::SB_WAVE);  // [T][64 lanes][CP]
  char* const ringx = smem + C::OFF_X;
  char* const ringa = smem + C::OFF_A;

  // ---- block -> (query block, slice); XCD-aware when S % 8 == 0 (slice s stays on one XCD)
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
  const int nsteps = nt * 2;
  const int nph = nt;  // 2-step phases
  const int pbase = qb * C::NQ + w * C::NCOL;

  if (*bad) {  // uniform over the grid: every wave leaves here
    for (int col = lane; col < C::NCOL; col += 64)
      if (pbase + col < nq) cand_cnt[(int64_t)(pbase + col) * S + s] = -1;
    return;
  }
  const float xnmax = __uint_as_float(*xnmax_bits);

  // query (B) fragments: lane (c, hh) of tile t holds hi(q')[16 ks + 8 hh .. +7] of column c
  bf16x8 bq[T][KS];
  float h[T];
  unsigned addr[T], lim[T], cap[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int p = pbase + t * 32 + c;
    const int q = p < nq ? qidx[p] : 0;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) bq[t][ks] = qhi[(q * KT + (ks >> 1)) * 4 + 2 * (ks & 1) + hh];
    addr[t] = (unsigned)(size_t)(sbuf + (t * 64 + lane) * C::CP);
    lim[t] = addr[t] + C::LIMN * 4;
    cap[t] = addr[t] + SUB * 4;  // the pad slot: appends saturate here
  }
  // the state of the column this lane owns in compactions: (tile hh, query c)
  const int own_p = pbase + hh * 32 + c;
  const bool own_valid = own_p < nq;
  int own_k = 0, own_flag = 0;
  float own_h = INFINITY, own_eps = 0.0f;
  if (own_valid) {
    const int q = qidx[own_p];
    own_k = qk[q];
    own_h = -FLT_MAX;
    own_eps = r1 * sqrtf(qn[q]) * sqrtf(xnmax) + r2 * xnmax;
  }
#pragma unroll
  for (int t = 0; t < T; ++t) h[t] = __shfl(own_h, t * 32 + c);
  // retire every compiler-issued load here: otherwise hipcc keeps them "pending" around the
  // phase loop and waits vmcnt at the loop's MFMAs, counting the hand-issued staging loads
  __builtin_amdgcn_s_waitcnt(0);

  // ---- staging: phase p = steps 2p, 2p+1 = 4 KT image pieces (step, 16-row half, kt) of 1 KiB
  // (hi halves; piece pc of phase p sits at ((4 KT p + pc) hl) KiB of the slice image).  The
  // wave stages bytes [w, w+1) * 512 KT of the phase and xinit[64 p + 8 w + lane], lane < 8.
  // The staging loads are inline asm with hand-counted vmcnt waits: hipcc's own wait
  // insertion drains vmcnt(0) at these loop-carried loads (a load two phases ahead would only
  // get one phase to land).  No other vector-memory access runs inside the phase loop.
  const char* const xbase = (const char*)(xfrag + (int64_t)t0 * (4 * KT * hl * 64));
  const char* const ibase = (const char*)(xinit + (int64_t)t0 * 64);
  const i32x4 xr = buffer_desc(xbase, nt * 4 * KT * hl * 1024);
  const i32x4 ir = buffer_desc(ibase, nt * 256);
  const int so = w * 512 * KT + lane * C::LDB;             // this lane's byte share of a phase
  const int sv = (((so >> 10) * hl) << 10) + (so & 1023);  // its hl-strided image offset
  const int xv_off = (lane < 8 ? 0 : 0x40000000) + 4 * (8 * w + lane);  // lanes >= 8: -> 0
  auto stage_load = [&](int p, Stage<KT>& st) __attribute__((always_inline)) {
    const int pl = p < nph ? p : nph - 1;  // past the end: re-read the last phase (never used)
    const int sa = pl * 4 * KT * hl * 1024, sx = pl * 256;
    if constexpr (KT == 1)
      asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(st.a) : "v"(sv), "s"(xr), "s"(sa));
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(st.a) : "v"(sv), "s"(xr), "s"(sa));
    asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(st.x) : "v"(xv_off), "s"(ir), "s"(sx));
  };
  // xinit point pi = 8 w + lane of the phase (step pi >> 5, row r = pi & 31) is C/D register
  // i = (r & 3) + 4 (r >> 3) of half (r >> 2) & 1: the ring holds [slot][half][16] fp32, so a
  // lane's whole C block is one 64-byte read
  const int xr_pi = 8 * w + (lane & 7), xr_r = xr_pi & 31;
  const int xs_off = (xr_pi >> 5) * 128 + ((xr_r >> 2) & 1) * 64 + ((xr_r & 3) + 4 * (xr_r >> 3)) * 4;
  // VMC = staged loads still allowed in flight (2 per younger staged phase)
  auto stage_store = [&](int p, Stage<KT>& st, auto vmc) __attribute__((always_inline)) {
    if constexpr (decltype(vmc)::value == 2)
      asm volatile("s_waitcnt vmcnt(2)" : "+v"(st.a), "+v"(st.x)::"memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(st.a), "+v"(st.x)::"memory");
    const int slot = (2 * p) & (C::RING - 1);
    *(typename Stage<KT>::A*)(ringa + slot * C::STEPB + so) = st.a;
    if (lane < 8) *(float*)(ringx + slot * 128 + xs_off) = st.x;
  };
  // consumer offsets inside a ring slot (hi-only image of the step: [rt][kt][64 x 16 B])
  int vo[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    vo[ks] = 16 * (((c >> 4) * KT + (ks >> 1)) * 64 + (2 * (ks & 1) + hh) * 16 + (c & 15));

  // ---- wave compaction: lane j owns column (t = hh, c)
  auto compact = [&](const bool final_pass) __attribute__((always_inline)) {
    int cnt[T];
#pragma unroll
    for (int t = 0; t < T; ++t)
      cnt[t] = (int)(addr[t] - (unsigned)(size_t)(sbuf + (t * 64 + lane) * C::CP)) >> 2;
    // counts of the owned column's two sub-buffers: (lane c, tile hh) and (lane c + 32, tile hh)
    const int a0 = __shfl(cnt[0], c), a1 = __shfl(cnt[1], c);
    const int b0n = __shfl(cnt[0], c + 32), b1n = __shfl(cnt[1], c + 32);
    const int n0 = hh ? a1 : a0, n1 = hh ? b1n : b0n;
    dmlp::wave_sync();
    // explicit LDS pointers: generic ones would compile to flat loads, which wait on vmcnt too
    lds_u32* const b0 = (lds_u32*)(size_t)(unsigned)(size_t)(sbuf + (hh * 64 + c) * C::CP);
    lds_u32* const b1 = (lds_u32*)(size_t)(unsigned)(size_t)(sbuf + (hh * 64 + c + 32) * C::CP);
    // a saturated sub-buffer (SUB appends) may have lost entries into its pad slot
    const int flag = own_flag | (n0 >= SUB) | (n1 >= SUB);
    float hc = own_h;
    // pass 1: ordered keys (0 = empty slot) packed as 15-bit pairs for the radix search
    unsigned mx = 0u;
    const unsigned mn = ord32(__float_as_uint(hc)) & 0xffff0000u;
    s16x2 pk[SUB];
#pragma unroll
    for (int v = 0; v < SUB; ++v) {
      const unsigned e0 = ord32(b0[v]) & (unsigned)((v - n0) >> 31);
      const unsigned e1 = ord32(b1[v]) & (unsigned)((v - n1) >> 31);
      mx = max(mx, max(e0, e1));
      pk[v] = __builtin_bit_cast(s16x2, (e0 >> 17) | ((e1 >> 17) << 16));
    }
    const bool sel = !flag && own_k >= 1 && n0 + n1 >= own_k;
    // k-th largest 16-bit key: radix search below the common prefix of [min, max] on 15-bit
    // keys packed two per register (screen_x1.hip); 2*T15 is a one-LSB lower bound
    const unsigned dif = (mx ^ mn) >> 17;
    const int top = (sel && dif) ? 31 - __clz((int)dif) : -1;
    unsigned Tk = mx >> 17;
    if (top >= 0) Tk &= ~((2u << top) - 1u);
    int topw = top;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int tt = __shfl_xor(topw, o);
      topw = tt > topw ? tt : topw;
    }
    for (int bit = topw; bit >= 0; --bit) {
      const short cand = (short)(Tk | (1u << bit));
      const s16x2 cc = {cand, cand};
      u16x2 lt = {0, 0};
#pragma unroll
      for (int v = 0; v < SUB; ++v) lt += __builtin_bit_cast(u16x2, pk[v] - cc) >> (unsigned short)15;
      const int ge = 2 * SUB - (int)lt.x - (int)lt.y;
      if (ge >= own_k) Tk |= 1u << bit;
    }
    Tk <<= 1;
    if (sel) {
      const float ak = __uint_as_float(unord32(Tk << 16));
      hc = fmaxf(hc, ak - 2.0f * own_eps);
    }
    const unsigned kh = flag ? 0xffffffffu : ord32(__float_as_uint(hc)) & 0xffff0000u;
    // pass 2: survivors.  Slots are visited interleaved (b0[0], b1[0], b0[1], ...): slot
    // (sub-buffer u, index i) has visit number 2 i + u, and the pos-th survivor goes to the slot
    // with visit number pos <= the current one, i.e. one already read (in place, no copy).
    if (!final_pass) {
      int pos = 0;
#pragma unroll 2
      for (int v = 0; v < 2 * SUB; ++v) {
        const unsigned raw = ((v & 1) ? b1 : b0)[v >> 1];
        const int nv = (v & 1) ? n1 : n0;
        const bool keep = (v >> 1) < nv && ord32(raw) >= kh;
        lds_u32* const dst = keep ? ((pos & 1) ? b1 : b0) + (pos >> 1) : b0 + SUB;
        *dst = raw;
        pos += keep ? 1 : 0;
      }
      const bool ovf = flag || pos > C::CAPE;
      own_flag = ovf ? 1 : 0;
      own_h = ovf ? INFINITY : hc;
      const int k0 = ovf ? 0 : (pos + 1) >> 1, k1 = ovf ? 0 : pos >> 1;
      dmlp::wave_sync();
      // back to the appenders: lane l's sub-buffer of tile t belongs to owner (t, l & 31)
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int src = t * 32 + c;
        const int f0 = __shfl(k0, src), f1 = __shfl(k1, src);
        addr[t] = (unsigned)(size_t)(sbuf + (t * 64 + lane) * C::CP) + 4u * (unsigned)(hh ? f1 : f0);
        h[t] = __shfl(own_h, src);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): resolve here, not at every later step
    } else if (own_valid) {
      int* const out = cand_ids + ((int64_t)own_p * S + s) * kX2IdCap;
      int kept = 0;
#pragma unroll 2
      for (int v = 0; v < 2 * SUB; ++v) {
        const unsigned raw = ((v & 1) ? b1 : b0)[v >> 1];
        const int nv = (v & 1) ? n1 : n0;
        const unsigned o = ord32(raw);
        const bool keep = (v >> 1) < nv && o >= kh;
        if (keep && kept < C::CAPE) out[kept] = (int)((o & 0xffff0000u) | (raw & 0xffffu));
        kept += keep ? 1 : 0;
      }
      cand_cnt[(int64_t)own_p * S + s] = (flag || kept > C::CAPE) ? -1 : kept;
      cand_h[2 * ((int64_t)own_p * S + s)] = hc;
      cand_h[2 * ((int64_t)own_p * S + s) + 1] = own_eps;
    }
  };

  f32x16 acc[2][T];
  unsigned long long trig = 0;  // wave-uniform: some sub-buffer passed its limit
  unsigned long long dbg_taken = 0, dbg_app = 0, dbg_comp = 0, dbg_ccyc = 0, dbg_bcyc = 0;
  // Compactions are workgroup events: a wave whose sub-buffer passed LIMN raises the event flag
  // of the next phase; after that phase's barrier every wave with a sub-buffer at least half
  // way to LIMN compacts, so the waves compact together instead of one at a time while the
  // other seven wait at the next barrier.  Flags rotate over 3 words: phase p reads flag p % 3,
  // raises (p + 1) % 3 and clears (p + 2) % 3 (read at p - 1, raised again only during p + 1).
  volatile int* const evf = (volatile int*)(smem + C::OFF_F);
  if (!PW && threadIdx.x < 3) evf[threadIdx.x] = 0;  // ordered before the first phase's barrier
  auto event = [&](int p) __attribute__((always_inline)) {
    const int ev = evf[p % 3];
    if (w == 0 && lane == 0) evf[(p + 2) % 3] = 0;
    if (ev) {
      bool half = false;
#pragma unroll
      for (int t = 0; t < T; ++t) half |= addr[t] + (C::LIMN / 2) * 4 > lim[t];
      if (__ballot(half)) {
        const unsigned long long t0c = (MODE & 8) ? __builtin_amdgcn_s_memtime() : 0;
        compact(false);
        if (MODE & 8) { ++dbg_comp; dbg_ccyc += __builtin_amdgcn_s_memtime() - t0c; }
      }
    }
  };
  auto raise = [&](int p) __attribute__((always_inline)) {
    if (trig && lane == 0) evf[(p + 1) % 3] = 1;
    trig = 0;
  };
  // step operands, read one step ahead: phase p + 1 is complete in the ring at barrier p
  struct Ops {
    bf16x8 a[KS];
    f32x16 cn;
  };
  auto read_ops = [&](int j, Ops& o) __attribute__((always_inline)) {
    if (MODE & 32) {  // ablation: operands stay in registers (no LDS reads)
      if (j < 2) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) o.a[ks] = bq[0][ks];
        const f32x16 z = {0.f};
        o.cn = z;
      }
      return;
    }
    const char* slot = ringa + (j & (C::RING - 1)) * C::STEPB;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) o.a[ks] = *(const bf16x8*)(slot + vo[ks]);
    if (MODE & 16) {
      const f32x16 z = {0.f};
      o.cn = z;
    } else {
      o.cn = *(const f32x16*)(ringx + (j & (C::RING - 1)) * 128 + hh * 64);
    }
  };
  auto mfma_step = [&](const Ops& o, f32x16(&ac)[T]) __attribute__((always_inline)) {
    const bf16x8* a = o.a;
    const f32x16 cn = o.cn;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bq[t][0], cn, 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks)
        ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks], bq[t][ks], ac[t], 0, 0, 0);
    }
  };
  auto epilogue = [&](int j, const f32x16(&ac)[T]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const f32x16 v = ac[t];
      float m[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        m[u] = fmaxf(fmaxf(fmaxf(v[4 * u], v[4 * u + 1]), v[4 * u + 2]), v[4 * u + 3]);
      const float M = fmaxf(fmaxf(fmaxf(m[0], m[1]), m[2]), m[3]);
      if (MODE & 4) {
        asm volatile("" ::"v"(v[0]), "v"(v[15]));
      } else if (MODE & 1) {
        asm volatile("" ::"v"(M));
      } else if (__ballot(M >= h[t])) {
        if (MODE & 8) ++dbg_taken;
        const unsigned g = (unsigned)(8 * j + hh);
        if (MODE & 64) {  // exec-masked appends (A/B: branches per run)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (m[u] >= h[t]) {
              *(__attribute__((address_space(3))) unsigned*)(size_t)addr[t] =
                  (__float_as_uint(m[u]) & 0xffff0000u) | (g + 2u * u);
              addr[t] = min(addr[t] + 4u, cap[t]);
              if (MODE & 8) ++dbg_app;
            }
          }
        } else {
          // branch-free: every lane writes each run's entry at its next free slot and advances
          // only on a hit (a miss is overwritten later and never read); the slot index
          // saturates at the pad slot
          unsigned a = addr[t];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            *(__attribute__((address_space(3))) unsigned*)(size_t)a =
                (__float_as_uint(m[u]) & 0xffff0000u) | (g + 2u * u);
            a += m[u] >= h[t] ? 4u : 0u;
            if (MODE & 8) dbg_app += m[u] >= h[t] ? 1 : 0;
          }
          addr[t] = min(a, cap[t]);
        }
        trig |= __ballot(addr[t] > lim[t]);
      }
    }
  };

  if constexpr (PW) {
    // ---- per-wave streaming (no LDS ring, no barrier): every wave loads its own steps from
    // L2 into a 4-deep register ring; C from one xinit value per lane + 16 DPP broadcasts
    if (nsteps > 0) {
      const int STEPG = 2 * KT * hl * 1024;  // global image bytes per step
      const __amdgpu_buffer_rsrc_t xrw = __builtin_amdgcn_make_buffer_rsrc(
          (void*)xbase, (short)0, nt * 4 * KT * hl * 1024, 0x00020000);
      const __amdgpu_buffer_rsrc_t irw = __builtin_amdgcn_make_buffer_rsrc(
          (void*)ibase, (short)0, nt * 256, 0x00020000);
      int vg[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        vg[ks] = 16 * ((((c >> 4) * KT + (ks >> 1)) * hl) * 64 + (2 * (ks & 1) + hh) * 16 + (c & 15));
      // lane 16 g + i reads row (i & 3) + 8 (i >> 2) + 4 hh: C/D register i of its half
      struct OpsW {
        bf16x8 a[KS];
      };
      auto read_w = [&](int j, OpsW& o) __attribute__((always_inline)) {
        const int jj = j < nsteps ? j : nsteps - 1;  // past the end: re-read (never used)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          o.a[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(xrw, vg[ks], jj * STEPG, 0));
      };
      // C ring: window w = steps 4w .. 4w + 3 (128 row terms) in LDS slot w & 1; lane L moves
      // row terms L and L + 64 of a window, one window ahead of its first read (no VALU: the
      // DPP broadcast of one value per lane into the 16-register C block cost 16 VALU per step)
      const unsigned xrb = (unsigned)C::SB_WAVE;  // LDS byte offset of the ring
      auto xpos = [](int f) {  // byte offset of window row term f in its slot
        const int sw = f >> 5, r = f & 31;
        return sw * 128 + ((r >> 2) & 1) * 64 + ((r & 3) + 4 * (r >> 3)) * 4;
      };
      const unsigned xp0 = (unsigned)xpos(lane), xp1 = (unsigned)xpos(lane + 64);
      auto xload = [&](int win, float& v0, float& v1) __attribute__((always_inline)) {
        v0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(irw, lane * 4, win * 512, 0));
        v1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(irw, lane * 4 + 256, win * 512, 0));
      };
      auto xstore = [&](int win, float v0, float v1) __attribute__((always_inline)) {
        const unsigned base = xrb + (unsigned)(win & 1) * 512u;
        *(__attribute__((address_space(3))) float*)(size_t)(base + xp0) = v0;
        *(__attribute__((address_space(3))) float*)(size_t)(base + xp1) = v1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the ring reads stay after it
      };
      auto cread = [&](int j) __attribute__((always_inline)) {
        return *(__attribute__((address_space(3))) const f32x16*)(size_t)(
            xrb + (unsigned)((j >> 2) & 1) * 512u + (unsigned)(j & 3) * 128u + (unsigned)hh * 64u);
      };
      auto mfma_w = [&](const OpsW& o, const f32x16& cn, f32x16(&ac)[T]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
          ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.a[0], bq[t][0], cn, 0, 0, 0);
#pragma unroll
          for (int ks = 1; ks < KS; ++ks)
            ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.a[ks], bq[t][ks], ac[t], 0, 0, 0);
        }
      };
      float xw0, xw1;
      {
        float v0, v1;
        xload(0, v0, v1);
        xstore(0, v0, v1);
      }
      xload(1, xw0, xw1);
      OpsW ring[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) read_w(r, ring[r]);
      f32x16 cn = cread(0);  // one block live: read after the previous step's epilogue
      const unsigned long long tl0 = (MODE & 8) ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll 1
      for (int j0 = 0; j0 < nsteps; j0 += 4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = j0 + r;
          if (r == 0) {
            // window j0/4 + 1 into the slot window j0/4 - 1 used (all its reads are done)
            xstore((j0 >> 2) + 1, xw0, xw1);
            xload((j0 >> 2) + 2, xw0, xw1);
          }
          if (j < nsteps) mfma_w(ring[r], cn, acc[r & 1]);
          read_w(j + 4, ring[r]);
          if (j > 0 && j - 1 < nsteps) epilogue(j - 1, acc[(r + 1) & 1]);
          if (r & 1) {  // every 2 steps (LIMN leaves room for 2 steps of appends)
            if (trig) {
              const unsigned long long t0c = (MODE & 8) ? __builtin_amdgcn_s_memtime() : 0;
              compact(false);
              if (MODE & 8) { ++dbg_comp; dbg_ccyc += __builtin_amdgcn_s_memtime() - t0c; }
            }
            trig = 0;
          }
          cn = cread(j + 1);  // the next step's C block (past the end: a stale window, unused)
        }
      }
      if ((nsteps & 3) == 0) {
        bool over = false;
#pragma unroll
        for (int t = 0; t < T; ++t) over |= addr[t] > lim[t];
        if (__ballot(over)) compact(false);
        epilogue(nsteps - 1, acc[1]);
      }
      if (MODE & 8) {
        const unsigned long long tl = __builtin_amdgcn_s_memtime() - tl0;
        unsigned long long v[6] = {dbg_taken, dbg_app, dbg_comp, dbg_ccyc, dbg_bcyc, tl};
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[1] += __shfl_xor(v[1], o);
        if (lane == 0)
#pragma unroll
          for (int i = 0; i < 6; ++i) atomicAdd(&g_x2_dbg[i], v[i]);
      }
    }
  } else if (nsteps > 0) {
    // prologue: phases 0 and 1 into the ring, phases 2 / 3 staged in registers (sx holds the
    // even phases, sy the odd ones: every staged load has two phases to land, with no copies)
    Stage<KT> sx, sy;
    using V0 = std::integral_constant<int, 0>;
    using V2 = std::integral_constant<int, 2>;
    stage_load(0, sx);
    stage_load(1, sy);
    stage_store(0, sx, V2{});
    stage_store(1, sy, V0{});
    stage_load(2, sx);
    stage_load(3, sy);
    const unsigned long long tl0 = (MODE & 8) ? __builtin_amdgcn_s_memtime() : 0;
    Ops o0, o1;
    auto phase = [&](int p, Stage<KT>& st) __attribute__((always_inline)) {
      const unsigned long long tb0 = (MODE & 8) ? __builtin_amdgcn_s_memtime() : 0;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (!(MODE & 2)) __builtin_amdgcn_s_barrier();  // phases p, p + 1 complete; all done with p - 1
      if (MODE & 8) dbg_bcyc += __builtin_amdgcn_s_memtime() - tb0;
      event(p);
      if (p == 0) read_ops(0, o0);
      // phase p + 2 (loaded at p - 2) -> the ring slots of p - 2; phase p + 4 -> registers
      stage_store(p + 2, st, V2{});  // the older of the two staged phases
      stage_load(p + 4, st);
      const int j0 = 2 * p;
      read_ops(j0 + 1, o1);
      mfma_step(o0, acc[0]);
      if (j0 > 0) epilogue(j0 - 1, acc[1]);
      if (j0 + 2 < nsteps) read_ops(j0 + 2, o0);
      mfma_step(o1, acc[1]);
      epilogue(j0, acc[0]);
      raise(p);
    };
#pragma unroll 1
    for (int p = 0; p < nph; p += 2) {
      phase(p, sx);
      if (p + 1 < nph) phase(p + 1, sy);
    }
    // the last phase's appends may have passed a limit: no barriers from here on, so the wave
    // compacts alone before the final step's epilogue
    {
      bool over = false;
#pragma unroll
      for (int t = 0; t < T; ++t) over |= addr[t] > lim[t];
      if (__ballot(over)) compact(false);
    }
    epilogue(nsteps - 1, acc[1]);  // nsteps = 2 nph: the last step is odd
    if (MODE & 8) {
      const unsigned long long tl = __builtin_amdgcn_s_memtime() - tl0;
      // per-lane tallies summed over the wave, one atomic per counter and wave
      unsigned long long v[6] = {dbg_taken, dbg_app, dbg_comp, dbg_ccyc, dbg_bcyc, tl};
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v[1] += __shfl_xor(v[1], o);
      if (lane == 0)
#pragma unroll
        for (int i = 0; i < 6; ++i) atomicAdd(&g_x2_dbg[i], v[i]);
    }
  }
  compact(true);
}

template <int KT, int SUB, bool PW>
int launch_x2(int hl, const void* xfrag, const float* xinit, int64_t n_tiles, const void* qhi,
              const float* qn, const int* qidx, const int* qk, int nq, const unsigned* xnmax,
              const unsigned* bad, float r1, float r2, int S, int* cand_ids, int* cand_cnt,
              float* cand_h, hipStream_t stream) {
  using C = X2Cfg<KT, SUB, PW>;
  const int n_qblocks = (nq + C::NQ - 1) / C::NQ;
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S;
  if (grid <= 0) return 0;
  static bool attr = false;  // > 64 KiB of dynamic LDS per workgroup
  if (!attr) {
    for (const void* f : {(const void*)k_screen_x2<KT, SUB, 0, PW>, (const void*)k_screen_x2<KT, SUB, 1, PW>,
                          (const void*)k_screen_x2<KT, SUB, 8, PW>, (const void*)k_screen_x2<KT, SUB, 64, PW>})
      hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
#define DMLP_X2_LAUNCH(M)                                                                        \
  hipLaunchKernelGGL((k_screen_x2<KT, SUB, M, PW>), dim3((unsigned)grid), dim3(64 * C::W), C::LDS, \
                     stream, (const u32x4*)xfrag, xinit, (int)n_tiles, (const bf16x8*)qhi, qn,   \
                     qidx, qk, nq, xnmax, bad, r1, r2, S, tps, n_qblocks, hl, cand_ids, cand_cnt, \
                     cand_h)
  switch (g_x2_mode) {  // ablations (timing only)
    case 1: DMLP_X2_LAUNCH(1); break;
    case 8: DMLP_X2_LAUNCH(8); break;
    case 64: DMLP_X2_LAUNCH(64); break;
    default: DMLP_X2_LAUNCH(0); break;
  }
#undef DMLP_X2_LAUNCH
  DMLP_LAUNCH_CHECK();
  return 0;
}

int g_x2_pw = 1;  // 1: per-wave streaming kernel, 0: 8-wave LDS-ring workgroups

constexpr int kX2Sub1 = 32, kX2Sub2 = 28;  // KT = 1 / 2 (LDS: the KT = 2 ring is twice as big)

}  // namespace

extern "C" int dmlp_screen_x2_kmax(void) { return 16; }
extern "C" int dmlp_screen_x2_qw(int KT) {
  if (KT != 1 && KT != 2) return 0;
  return g_x2_pw ? X2Cfg<1, kX2Sub1, true>::NQ : X2Cfg<1, kX2Sub1>::NQ;
}
extern "C" void dmlp_set_x2_pw(int on) { g_x2_pw = on ? 1 : 0; }
extern "C" int dmlp_screen_x2_cap(int kmax) { (void)kmax; return kX2IdCap; }
// workgroups per CU: 8 single-wave ones (per-wave form), or one of 8 waves (the LDS holds one)
extern "C" int dmlp_screen_x2_waves_per_cu(int kmax) { (void)kmax; return g_x2_pw ? 8 : 1; }
extern "C" void dmlp_set_x2_mode(int mode) { g_x2_mode = mode; }
extern "C" int dmlp_x2_debug_counters(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x2_dbg), sizeof(g_x2_dbg));
  if (e != hipSuccess) return -(int)e;
  if (reset) {
    unsigned long long z[8] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_x2_dbg), z, sizeof(z));
    if (e != hipSuccess) return -(int)e;
  }
  return 0;
}

extern "C" int dmlp_screen_x2(int KT, int hl, int A, const void* xfrag, const float* xinit,
                              int64_t n_tiles, int64_t n_points, const void* qhi, const float* qn,
                              const int* qidx, const int* qk, int nq, int kmax,
                              const unsigned* xnmax_bits, const unsigned* bad, int S,
                              int* cand_ids, int* cand_cnt, float* cand_h, void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || n_tiles < 0 || n_tiles > 0x7fffffff / 64 || n_points > n_tiles * 64) return -1;
  if ((n_tiles + S - 1) / S > 4096) return -4;  // 16-bit group index per slice
  if (kmax > dmlp_screen_x2_kmax() || KT < 1 || KT > 2 || A > KT * 32) return -3;
  if (hl != 1 && hl != 2) return -1;
  float r1, r2;
  dmlp_screen_x1_bound(A, &r1, &r2);
  hipStream_t st = (hipStream_t)stream;
#define DMLP_X2_ARGS hl, xfrag, xinit, n_tiles, qhi, qn, qidx, qk, nq, xnmax_bits, bad, r1, r2, S, \
                     cand_ids, cand_cnt, cand_h, st
  if (g_x2_pw)
    return KT == 1 ? launch_x2<1, kX2Sub1, true>(DMLP_X2_ARGS) : launch_x2<2, kX2Sub2, true>(DMLP_X2_ARGS);
  return KT == 1 ? launch_x2<1, kX2Sub1, false>(DMLP_X2_ARGS) : launch_x2<2, kX2Sub2, false>(DMLP_X2_ARGS);
#undef DMLP_X2_ARGS
}
