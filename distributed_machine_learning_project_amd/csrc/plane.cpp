// plane.cpp — the node render plane: P ranks of one node stepping against ONE dataset share its
// host render instead of each rendering all of it.
//
// bench_4 replicates the whole dataset to every rank (one MPI_Bcast, bench_4 @0xc199).  On an
// MI355X node every rank's step needs the same per-call products of it: the fp16 tile image +
// norms the screen reads, and the lossless int32 rows the exact re-rank reads (pipeline.hip).
// Rendered by every rank, that is P times the same host work and host-memory traffic (the P-rank
// farm's host budget, profiles/r7h_host_budget.md).  Here the dataset is cut into slices (the
// early start's image slices, pipeline.hip kEarlySlices); ranks [0, renderers) render them
// round-robin ONCE into a node-shared page-locked segment, each slice published by a generation
// flag, and every rank's step copies the slices from the segment over its own PCIe link
// (pipeline.hip Step, plane mode).  renderers = 1 is the engine.h drop-in at P > 1: only rank 0
// holds the harness's vectors (common.cpp:93-117), so it renders for everyone.
//
// Segment: [header 64 KiB | fp16 image | xinit | int32 rows | fp64 rows (with_f64)].  Flags are
// gen << 2 | bits, written with release stores after the slice's bytes and read with acquire
// loads, so a consumer that sees its call's generation sees the slice.  Generations increase per
// call and the callers separate calls by a barrier of all plane ranks (every front end's report
// egress has one), so a slice is never re-rendered while another rank still copies it.
#include "dmlp.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>

#include <immintrin.h>

namespace {

constexpr uint64_t kMagic = 0x646d6c70706c6e31ull;  // "dmlppln1"
constexpr int kMaxSlices = 64;

struct Hdr {
  uint64_t magic;
  int64_t N, A, ns, with_f64;
  alignas(64) int64_t mu_flag;
  double mu[256];
  alignas(64) int64_t img_flag[kMaxSlices];
  int64_t row_flag[kMaxSlices];
  float nmax[kMaxSlices];
};
static_assert(sizeof(Hdr) <= 65536, "plane header");

struct Layout {
  int64_t nt = 0, W = 0, rt = 1;
  int ns = 0, KT = 1;
  int64_t off_img = 0, off_xin = 0, off_r32 = 0, off_r64 = 0, total = 0;
};

int64_t up(int64_t b) { return (b + 4095) & ~int64_t(4095); }

Layout layout(int64_t N, int A, int with_f64) {
  Layout L;
  L.KT = dmlp_screen_kt(A);
  L.W = (int64_t)L.KT * 32;
  L.nt = (N + 63) / 64;
  L.ns = (int)std::min<int64_t>(dmlp_plane_slices(), std::max<int64_t>(L.nt, 1));
  L.rt = std::max<int64_t>(1, (L.nt + L.ns - 1) / L.ns);
  L.off_img = 65536;
  L.off_xin = L.off_img + up(L.nt * 64 * L.W * 2);
  L.off_r32 = L.off_xin + up(L.nt * 64 * 4);
  L.off_r64 = L.off_r32 + up(N * A * 4);
  L.total = L.off_r64 + (with_f64 ? up(N * A * 8) : 0);
  return L;
}

int64_t load_acq(const int64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
void store_rel(int64_t* p, int64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

Hdr* hdr(const dmlp_plane* p) { return (Hdr*)p->base; }

// the plane must describe this dataset (every rank passes the same N, A)
bool valid(const dmlp_plane* p, int64_t N, int A) {
  if (!p || !p->base || p->gen <= 0 || N < 0 || A < 1 || A > 256) return false;
  const Layout L = layout(N, A, p->with_f64);
  return p->bytes >= L.total;
}

double wait_bound_s(const dmlp_plane* p) { return p->wait_s > 0 ? p->wait_s : 60.0; }

// spin on *f until it reaches gen (acquire): short pause loop, then yields; false on timeout
bool wait_flag(const dmlp_plane* p, const int64_t* f, int64_t* out) {
  const int64_t want = p->gen;
  int64_t v = load_acq(f);
  if ((v >> 2) == want) {
    *out = v;
    return true;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; ++spin) {
    v = load_acq(f);
    if ((v >> 2) == want) {
      *out = v;
      return true;
    }
    if ((v >> 2) > want) return false;  // a later call's flag: the ranks' generations diverged
    if (spin < 2048) {
      _mm_pause();
    } else {
      std::this_thread::yield();
      if ((spin & 1023) == 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >
              wait_bound_s(p))
        return false;
    }
  }
}

}  // namespace

extern "C" int dmlp_plane_slices(void) { return 8; }

extern "C" int64_t dmlp_plane_bytes(int64_t N, int A, int with_f64) {
  if (N < 0 || A < 1 || A > 256) return -1;
  return layout(N, A, with_f64).total;
}

extern "C" int dmlp_plane_slice(int64_t N, int A, int i, int64_t* t0, int64_t* t1) {
  const Layout L = layout(N, A, 0);
  if (i < 0 || i >= L.ns) return -1;
  *t0 = std::min<int64_t>(L.nt, (int64_t)i * L.rt);
  *t1 = std::min<int64_t>(L.nt, *t0 + L.rt);
  return L.ns;
}

extern "C" int dmlp_plane_init(void* base, int64_t bytes, int64_t N, int A, int with_f64) {
  if (!base) return -1;
  const Layout L = layout(N, A, with_f64);
  if (bytes < L.total) return -2;
  Hdr* h = (Hdr*)base;
  std::memset(h, 0, sizeof(Hdr));
  h->N = N;
  h->A = A;
  h->ns = L.ns;
  h->with_f64 = with_f64;
  __atomic_store_n(&h->magic, kMagic, __ATOMIC_RELEASE);
  return 0;
}

extern "C" int dmlp_plane_regions(const dmlp_plane* p, int64_t N, int A, void** img, void** xin,
                                  void** r32, void** r64) {
  if (!valid(p, N, A)) return -1;
  const Layout L = layout(N, A, p->with_f64);
  char* b = (char*)p->base;
  if (img) *img = b + L.off_img;
  if (xin) *xin = b + L.off_xin;
  if (r32) *r32 = b + L.off_r32;
  if (r64) *r64 = p->with_f64 ? (void*)(b + L.off_r64) : nullptr;
  return 0;
}

// mu (plane rank 0): the centre of the first min(N, 4096) rows, published for every rank's
// query and image render — every rank must centre with the SAME bits
extern "C" int dmlp_plane_put_mu(const dmlp_plane* p, int A, const double* mu) {
  if (!p || !p->base || A < 1 || A > 256) return -1;
  Hdr* h = hdr(p);
  std::memcpy(h->mu, mu, sizeof(double) * A);
  store_rel(&h->mu_flag, p->gen << 2);
  return 0;
}
extern "C" int dmlp_plane_get_mu(const dmlp_plane* p, int A, double* mu) {
  if (!p || !p->base || A < 1 || A > 256) return -1;
  Hdr* h = hdr(p);
  int64_t f = 0;
  if (!wait_flag(p, &h->mu_flag, &f)) return -4;
  std::memcpy(mu, h->mu, sizeof(double) * A);
  return 0;
}

// Render dataset slice i (rows X row-major, or Xr row pointers): what = 1 the fp16 image tiles +
// xinit + the slice's max norm, what = 2 the slice's rows (lossless int32, else fp64 into the
// fp64 region when the plane has one — otherwise the consumers read the node-shared X).  Then
// publish the slice's flag.  Returns the flag bits (1: image outside the fp16 range, 2: fp64
// rows), or < 0.
extern "C" int dmlp_plane_render(const dmlp_plane* p, const double* X, const double* const* Xr,
                                 int64_t N, int A, const double* mu, int what, int i) {
  if (!valid(p, N, A) || (!X && !Xr)) return -1;
  const Layout L = layout(N, A, p->with_f64);
  if (i < 0 || i >= L.ns) return -1;
  Hdr* h = hdr(p);
  char* b = (char*)p->base;
  const int64_t t0 = std::min<int64_t>(L.nt, (int64_t)i * L.rt), t1 = std::min<int64_t>(L.nt, t0 + L.rt);
  int bits = 0;
  if (what == 1) {
    float m = 0.0f;
    uint16_t* img = (uint16_t*)(b + L.off_img);
    float* xin = (float*)(b + L.off_xin);
    const int bad = Xr ? dmlp_cpu_prep_data_tiles_rows(Xr, N, A, mu, L.KT, t0, t1, img, xin, &m)
                       : dmlp_cpu_prep_data_tiles(X, N, A, mu, L.KT, t0, t1, img, xin, &m);
    if (bad) {
      bits |= 1;
      m = INFINITY;
    }
    h->nmax[i] = m;
    store_rel(&h->img_flag[i], (p->gen << 2) | bits);
    return bits;
  }
  if (what == 2) {
    const int64_t r0 = std::min<int64_t>(N, t0 * 64), r1 = std::min<int64_t>(N, t1 * 64);
    int32_t* r32 = (int32_t*)(b + L.off_r32) + r0 * A;
    const int fail = r1 <= r0 ? 0
                     : Xr ? dmlp_cpu_rows_i32_rows(Xr + r0, r1 - r0, A, r32)
                          : dmlp_cpu_rows_i32(X + r0 * A, (r1 - r0) * A, r32);
    if (fail) {
      bits |= 2;
      if (p->with_f64) {
        double* r64 = (double*)(b + L.off_r64) + r0 * A;
        if (Xr) dmlp_cpu_gather_rows(Xr + r0, r1 - r0, A, r64);
        else std::memcpy(r64, X + r0 * A, sizeof(double) * (r1 - r0) * A);
      }
    }
    store_rel(&h->row_flag[i], (p->gen << 2) | bits);
    return bits;
  }
  return -1;
}

// Wait for slice i's flag of this call (what 1 image, 2 rows); *bits = its bits, *nmax = the
// image slice's max norm.  0, or -4 on timeout / a diverged generation.
extern "C" int dmlp_plane_wait(const dmlp_plane* p, int what, int i, int* bits, float* nmax) {
  if (!p || !p->base || i < 0 || i >= kMaxSlices || (what != 1 && what != 2)) return -1;
  Hdr* h = hdr(p);
  int64_t f = 0;
  if (!wait_flag(p, what == 1 ? &h->img_flag[i] : &h->row_flag[i], &f)) return -4;
  if (bits) *bits = (int)(f & 3);
  if (nmax) *nmax = h->nmax[i];
  return 0;
}

// Slice i's rows as fp64 in dst (the whole [N][A] array's slot of the slice): waits for the
// slice, then the int32 m / 1e6 (IEEE division: the exact input doubles, as the device's
// k_rows_from_i32) or the fp64 copy (the plane's region, else X: the node-shared rows).  The
// host consumers of the plane (the drop-in's CPU window farm).  0, -4 on timeout.
extern "C" int dmlp_plane_rows_f64(const dmlp_plane* p, int64_t N, int A, int i, const double* X,
                                   double* dst) {
  if (!valid(p, N, A)) return -1;
  const Layout L = layout(N, A, p->with_f64);
  if (i < 0 || i >= L.ns) return -1;
  int bits = 0;
  if (dmlp_plane_wait(p, 2, i, &bits, nullptr) != 0) return -4;
  const int64_t t0 = std::min<int64_t>(L.nt, (int64_t)i * L.rt), t1 = std::min<int64_t>(L.nt, t0 + L.rt);
  const int64_t r0 = std::min<int64_t>(N, t0 * 64), r1 = std::min<int64_t>(N, t1 * 64);
  const char* b = (const char*)p->base;
  if (bits & 2) {
    const double* src = p->with_f64 ? (const double*)(b + L.off_r64) : X;
    if (!src) return -1;
    std::memcpy(dst + r0 * A, src + r0 * A, sizeof(double) * (r1 - r0) * A);
  } else {
    const int32_t* src = (const int32_t*)(b + L.off_r32);
    for (int64_t e = r0 * A; e < r1 * A; ++e) dst[e] = (double)src[e] / 1.0e6;
  }
  return 0;
}

// Non-blocking: 1 when slice i's flag of this call is set, else 0.
extern "C" int dmlp_plane_ready(const dmlp_plane* p, int what, int i) {
  if (!p || !p->base || i < 0 || i >= kMaxSlices) return 0;
  Hdr* h = hdr(p);
  return (load_acq(what == 1 ? &h->img_flag[i] : &h->row_flag[i]) >> 2) == p->gen ? 1 : 0;
}
