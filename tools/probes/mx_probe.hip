// Probe of v_mfma_scale_f32_16x16x128_f8f6f4's block-scale lane map on gfx950 (run on the GPU box):
//   lane l holds row (l & 15) of A (column of B): K bytes [16g, 16g+16) in VGPRs 0-3 and
//   [64+16g, 64+16g+16) in VGPRs 4-7 (g = l >> 4), and its scale VGPR (byte 0 with opsel 0) is the
//   E8M0 scale of the CONTIGUOUS K-block [32g, 32g+32) of that row -- values held by lanes of other
//   groups (measured: mx_probe3.hip; the lane's own 32 bytes are NOT its block).
//   So MX blocks are 32 contiguous bytes of a K-major row and lane (16b + r) supplies block b's scale.
// Exact small-integer e4m3 data and power-of-two scales: every product is exact in fp32.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// A [16][128] e4m3, B [16][128] e4m3 (row j = column j of the product), sa/sb [16][4] E8M0;
// CHUNKS: 0 = lane loads bytes [32g, 32g+32), 1 = bytes [16g, 16g+16) and [64+16g, 64+16g+16)
template <int CHUNKS>
__global__ void probe(const uint8_t* A, const uint8_t* B, const uint8_t* sa, const uint8_t* sb, float* C) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  i32x8 a, b;
  const uint32_t* pa = reinterpret_cast<const uint32_t*>(A + r * 128);
  const uint32_t* pb = reinterpret_cast<const uint32_t*>(B + r * 128);
  for (int w = 0; w < 8; ++w) {
    const int byte = CHUNKS == 0 ? 32 * g + 4 * w : (w < 4 ? 16 * g + 4 * w : 64 + 16 * g + 4 * (w - 4));
    a[w] = (int)pa[byte / 4];
    b[w] = (int)pb[byte / 4];
  }
  const int ea = sa[r * 4 + g], eb = sb[r * 4 + g];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, ea, 0, eb);
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = acc[i];  // row 4*(l>>4)+i, col l&15
}

static uint8_t e4m3_of_int(int v) {  // exact small integers |v| <= 8
  if (v == 0) return 0;
  const uint8_t s = v < 0 ? 0x80 : 0;
  int m = std::abs(v), e = 0;
  while (m >= 2 << e) ++e;  // 2^e <= m < 2^(e+1)
  const int frac = ((m << 3) >> e) & 7;  // 3 mantissa bits
  return s | (uint8_t)((e + 7) << 3) | (uint8_t)frac;
}

int main() {
  uint8_t hA[16 * 128], hB[16 * 128], hsa[64], hsb[64];
  int iA[16 * 128], iB[16 * 128];
  srand(7);
  for (int i = 0; i < 16 * 128; ++i) {
    iA[i] = rand() % 9 - 4;
    iB[i] = rand() % 9 - 4;
    hA[i] = e4m3_of_int(iA[i]);
    hB[i] = e4m3_of_int(iB[i]);
  }
  for (int i = 0; i < 64; ++i) {
    hsa[i] = (uint8_t)(124 + rand() % 7);
    hsb[i] = (uint8_t)(124 + rand() % 7);
  }
  uint8_t *dA, *dB, *dsa, *dsb;
  float* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dsa, 64);
  hipMalloc(&dsb, 64);
  hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, 64, hipMemcpyHostToDevice);
  hipMemcpy(dsb, hsb, 64, hipMemcpyHostToDevice);
  int rc = 0;
  for (int chunks = 0; chunks < 2; ++chunks) {
    if (chunks == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
    else hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
    float hC[256];
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    // reference under the hypothesis: the block of lane (row, g) = the bytes that lane loaded
    int bad = 0;
    double maxerr = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double ref = 0;
        for (int g = 0; g < 4; ++g) {
          double s = 0;
          for (int t = 0; t < 32; ++t) {
            const int k = 32 * g + t;  // the natural block (chunks=0 loads it as a lane's own data: negative control)
            s += (double)iA[i * 128 + k] * iB[j * 128 + k];
          }
          ref += s * std::ldexp(1.0, hsa[i * 4 + g] - 127) * std::ldexp(1.0, hsb[j * 4 + g] - 127);
        }
        const double e = std::fabs(ref - hC[i * 16 + j]);
        if (e > 1e-6 * (1 + std::fabs(ref))) ++bad;
        if (e > maxerr) maxerr = e;
      }
    printf("chunks=%d (lane holds %s): mismatches %d / 256, max abs err %g%s\n", chunks,
           chunks == 0 ? "bytes [32g, 32g+32)" : "bytes [16g,+16) and [64+16g,+16)", bad, maxerr,
           chunks == 0 ? " (expected to mismatch)" : "");
    if (chunks == 1 && bad) rc = 1;
  }
  return rc;
}
