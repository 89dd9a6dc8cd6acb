// Probe (diagnostic): which (row, 32-k block) each lane's E8M0 scale of
// v_mfma_scale_f32_16x16x128_f8f6f4 applies to. A = 1, B[k][c] = 1 iff
// k/32 == c%4; doubling lane L's scale doubles exactly the (row, block)
// entries it owns. Prints the owner map for A (scale_a) and B (scale_b).
#include <hip/hip_runtime.h>

#include <cstdio>
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

int main() {
  const unsigned char one = 0x38;  // e4m3 1.0
  for (int which = 0; which < 2; ++which) {
    // which 0: A = 1, B block selector; which 1: B = 1, A block selector (A[r][k] = 1 iff k/32 == r%4)
    std::vector<unsigned char> ha(64 * 32), hb(64 * 32);
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int k = 32 * (l >> 4) + j, rc = l & 15;
        ha[l * 32 + j] = which == 0 ? one : ((k >> 5) == (rc & 3) ? one : 0);
        hb[l * 32 + j] = which == 1 ? one : ((k >> 5) == (rc & 3) ? one : 0);
      }
    unsigned char *da, *db;
    int *dsa, *dsb;
    v4f* dc;
    (void)hipMalloc(&da, 64 * 32);
    (void)hipMalloc(&db, 64 * 32);
    (void)hipMalloc(&dsa, 256);
    (void)hipMalloc(&dsb, 256);
    (void)hipMalloc(&dc, 64 * sizeof(v4f));
    (void)hipMemcpy(da, ha.data(), 64 * 32, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb.data(), 64 * 32, hipMemcpyHostToDevice);
    printf("%s scale owners (lane: entries doubled as [row-or-col, block])\n", which == 0 ? "A" : "B");
    for (int L = 0; L < 64; ++L) {
      std::vector<int> sa(64, 127), sb(64, 127);
      (which == 0 ? sa : sb)[L] = 128;
      (void)hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
      (void)hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, 0, (const v8i*)da, (const v8i*)db, dsa,
                         dsb, dc);
      std::vector<v4f> hc(64);
      (void)hipMemcpy(hc.data(), dc, 64 * sizeof(v4f), hipMemcpyDeviceToHost);
      printf("  lane %2d:", L);
      int cnt = 0;
      for (int l = 0; l < 64; ++l)
        for (int q = 0; q < 4; ++q) {
          const int c = l & 15, r = (l >> 4) * 4 + q;
          const float v = hc[l][q];
          if (v != 32.f) {
            // which 0: D[r][c] = 32 * sA(r, block c%4); which 1: D[r][c] = 32 * sB(c, block r%4)
            if (which == 0 && c < 4) { printf(" [r%d,b%d]=%g", r, c & 3, v); ++cnt; }
            if (which == 1 && r < 4) { printf(" [c%d,b%d]=%g", c, r & 3, v); ++cnt; }
          }
        }
      printf("%s\n", cnt ? "" : " (none)");
    }
  }
  return 0;
}
