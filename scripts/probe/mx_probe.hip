// Probe (diagnostic, not product code): the lane maps of gfx950's
// v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands and per-lane E8M0
// scales, and the rounding of v_cvt_pk_fp8_f32. Exact small-integer data, an
// ASYMMETRIC B, checked against a host reference. Build + run:
//   hipcc -O2 --offload-arch=gfx950 scripts/probe/mx_probe.hip -o /tmp/mx_probe && /tmp/mx_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void mfma_probe(const v8i* a, const v8i* b, const int* sa, const int* sb, v4f* c) {
  const int l = threadIdx.x;
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0,
                                                          sb[l]);
  c[l] = acc;
}

__global__ void cvt_probe(const float* f, int* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 < n) o[i] = __builtin_amdgcn_cvt_pk_fp8_f32(f[2 * i], f[2 * i + 1], 0, false);
}

// e4m3fn (OCP) encode of small integers
static unsigned char enc_int(int v) {
  if (v == 0) return 0;
  const unsigned s = v < 0 ? 0x80 : 0;
  int a = std::abs(v);
  int e = 0;
  while ((1 << (e + 1)) <= a) ++e;
  const int m = (a - (1 << e)) * 8 / (1 << e);  // exact for |v| <= 16
  return s | ((e + 7) << 3) | m;
}
static double dec(unsigned char b) {
  const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  double v = e == 0 ? m * std::ldexp(1.0, -9) : (1 + m / 8.0) * std::ldexp(1.0, e - 7);
  if (e == 15 && m == 7) v = NAN;
  return s ? -v : v;
}

int main() {
  // A[16][128], B[128][16] small integers in [-3, 3], B asymmetric
  int A[16][128], B[128][16];
  for (int r = 0; r < 16; ++r)
    for (int k = 0; k < 128; ++k) A[r][k] = ((r * 7 + k * 3 + (k >> 5)) % 7) - 3;
  for (int k = 0; k < 128; ++k)
    for (int c = 0; c < 16; ++c) B[k][c] = ((k * 5 + c * 11 + c * c) % 7) - 3;
  // lane map (found with mx_scale_probe): lane l holds row/col l&15; bytes 0..15 are
  // k = 16g + j, bytes 16..31 are k = 64 + 16g + (j - 16), g = l >> 4 (natural 16-B
  // chunks g and 4 + g of a 128-byte K row, as the f16 16x16x32 pair of k-steps).
  // Scale lane L applies to row/col L&15, k-block L>>4 (k 32*(L>>4) .. +31).
  auto kmap = [](int l, int j) { return j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + j - 16; };
  std::vector<unsigned char> ha(64 * 32), hb(64 * 32);
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      ha[l * 32 + j] = enc_int(A[l & 15][kmap(l, j)]);
      hb[l * 32 + j] = enc_int(B[kmap(l, j)][l & 15]);
    }
  int fails_total = 0;
  for (int mode = 0; mode < 3; ++mode) {
    // scales: mode 0 all 1.0; mode 1 A scale 2^(l>>4) per lane; mode 2 both vary per lane
    std::vector<int> sa(64), sb(64);
    for (int l = 0; l < 64; ++l) {
      sa[l] = 127 + (mode >= 1 ? ((l >> 4) + (l & 3)) % 3 - 1 : 0);
      sb[l] = 127 + (mode == 2 ? ((l >> 4) * 2 + (l & 15)) % 4 - 2 : 0);
    }
    unsigned char *da, *db;
    int *dsa, *dsb;
    v4f* dc;
    hipMalloc(&da, 64 * 32);
    hipMalloc(&db, 64 * 32);
    hipMalloc(&dsa, 256);
    hipMalloc(&dsb, 256);
    hipMalloc(&dc, 64 * sizeof(v4f));
    hipMemcpy(da, ha.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, 0, (const v8i*)da, (const v8i*)db, dsa,
                       dsb, dc);
    std::vector<v4f> hc(64);
    hipMemcpy(hc.data(), dc, 64 * sizeof(v4f), hipMemcpyDeviceToHost);
    // reference: D[r][c] = sum_k A[r][k] 2^(sa(lane of (r,kb))-127) B[k][c] 2^(sb(lane of (c,kb))-127)
    int fails = 0;
    for (int l = 0; l < 64; ++l)
      for (int q = 0; q < 4; ++q) {
        const int c = l & 15, r = (l >> 4) * 4 + q;  // C layout: col = lane&15, row = 4*(lane>>4)+reg
        double ref = 0;
        for (int k = 0; k < 128; ++k) {
          const int kb = k >> 5;
          ref += A[r][k] * std::ldexp(1.0, sa[kb * 16 + r] - 127) * B[k][c] *
                 std::ldexp(1.0, sb[kb * 16 + c] - 127);
        }
        if (std::fabs(ref - hc[l][q]) > 1e-6) {
          if (fails < 4) printf("mode %d mismatch r=%d c=%d got %g want %g\n", mode, r, c, hc[l][q], ref);
          ++fails;
        }
      }
    printf("mfma_scale 16x16x128 fp8 mode %d: %s (%d mismatches)\n", mode, fails ? "FAIL" : "PASS", fails);
    fails_total += fails;
  }
  // cvt_pk_fp8_f32: rounding vs RNE to e4m3fn, and out-of-range behaviour
  std::vector<float> f;
  for (int i = 0; i < 4000; ++i) f.push_back((float)((i - 2000) * 0.137 + 0.01 * std::sin(i)));
  for (int i = 0; i < 400; ++i) f.push_back(std::ldexp(1.0f + i / 400.f, -12 + i % 16));
  f.push_back(448.f); f.push_back(464.f); f.push_back(470.f); f.push_back(1000.f);
  f.push_back(-500.f); f.push_back(0.f);
  if (f.size() % 2) f.push_back(1.f);
  const int n = (int)f.size();
  float* df;
  int* dout;
  hipMalloc(&df, n * 4);
  hipMalloc(&dout, n * 2);
  hipMemcpy(df, f.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(cvt_probe, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, df, dout, n);
  std::vector<int> ho(n / 2);
  hipMemcpy(ho.data(), dout, n * 2, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const unsigned char b = (ho[i / 2] >> (8 * (i & 1))) & 0xff;
    const double x = f[i];
    if (std::fabs(x) > 448) {
      printf("cvt %g -> 0x%02x (%g)\n", x, b, dec(b));
      continue;
    }
    // nearest representable, ties to even mantissa
    double best = 1e30;
    int bb = -1;
    for (int c = 0; c < 256; ++c) {
      const double v = dec((unsigned char)c);
      if (std::isnan(v)) continue;
      const double d = std::fabs(v - x);
      if (d < best - 1e-300 || (d == best && bb >= 0 && (c & 1) == 0 && (c & 0x7f) != 0)) {
        if (!(d == best && (bb & 1) == 0)) { best = d; bb = c; }
      }
    }
    if (std::fabs(dec(b) - x) > best * (1 + 1e-12) + 1e-300) {
      if (bad < 6) printf("cvt %.9g -> %g (0x%02x), nearest %g\n", x, dec(b), b, dec(bb));
      ++bad;
    }
  }
  printf("cvt_pk_fp8_f32: %s (%d of %d not nearest)\n", bad ? "FAIL" : "PASS", bad, n);
  return fails_total || bad;
}
