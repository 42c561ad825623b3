// Probe: v_dot2c_f32_f16 vs cvt + fma on fp16 pairs (subnormal inputs, rounding), one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdlib>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned* a, const unsigned* b, const float* c, float* d2, float* fm, int n) {
  int i = threadIdx.x + blockIdx.x * blockDim.x;
  if (i >= n) return;
  const unsigned x = a[i], y = b[i];
  d2[i] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, x), __builtin_bit_cast(h2, y), c[i], false);
  float s = c[i];
  s = __builtin_fmaf((float)__builtin_bit_cast(_Float16, (unsigned short)(x & 0xffff)),
                     (float)__builtin_bit_cast(_Float16, (unsigned short)(y & 0xffff)), s);
  s = __builtin_fmaf((float)__builtin_bit_cast(_Float16, (unsigned short)(x >> 16)),
                     (float)__builtin_bit_cast(_Float16, (unsigned short)(y >> 16)), s);
  fm[i] = s;
}
static float h2f(unsigned short h) { _Float16 v; __builtin_memcpy(&v, &h, 2); return (float)v; }
int main() {
  const int n = 1 << 16;
  unsigned *a, *b; float *c, *d2, *fm;
  hipMallocManaged(&a, n * 4); hipMallocManaged(&b, n * 4); hipMallocManaged(&c, n * 4);
  hipMallocManaged(&d2, n * 4); hipMallocManaged(&fm, n * 4);
  srand(1);
  for (int i = 0; i < n; ++i) {
    unsigned short r[4];
    for (int j = 0; j < 4; ++j) r[j] = (unsigned short)(rand() & 0x7fff);
    if (i % 4 == 0) { r[0] &= 0x03ff; }           // subnormal operand
    if (i % 8 == 1) { r[0] = 0x3c00; r[2] = 0x0001; r[1] = 0; r[3] = 0; }  // 1 * smallest subnormal
    if (rand() & 1) r[1] |= 0x8000;
    a[i] = r[0] | (unsigned)r[1] << 16; b[i] = r[2] | (unsigned)r[3] << 16;
    c[i] = (i % 3 == 0) ? 0.0f : (float)((rand() % 2000) - 1000) * 0.37f;
  }
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, a, b, c, d2, fm, n);
  hipDeviceSynchronize();
  int diff = 0, worse = 0, sub_flush = 0;
  double maxrel_d = 0, maxrel_f = 0;
  for (int i = 0; i < n; ++i) {
    const double ex = (double)h2f(a[i] & 0xffff) * h2f(b[i] & 0xffff) + (double)h2f(a[i] >> 16) * h2f(b[i] >> 16) + c[i];
    const double ed = fabs(d2[i] - ex), ef = fabs(fm[i] - ex);
    if (d2[i] != fm[i]) ++diff;
    if (ed > ef) ++worse;
    const double sc = fabs(ex) + 1e-30;
    if (ed / sc > maxrel_d) maxrel_d = ed / sc;
    if (ef / sc > maxrel_f) maxrel_f = ef / sc;
    if (i % 8 == 1 && c[i] == 0.0f && d2[i] == 0.0f) ++sub_flush;
  }
  printf("n %d  dot2!=fma %d  dot2 worse %d  max rel err dot2 %.3e fma %.3e  subnormal products flushed %d\n",
         n, diff, worse, maxrel_d, maxrel_f, sub_flush);
  for (int i = 0; i < 16; ++i)
    if (d2[i] != fm[i]) printf("  i %d a %08x b %08x c %g dot2 %.9g fma %.9g\n", i, a[i], b[i], c[i], d2[i], fm[i]);
  return 0;
}
