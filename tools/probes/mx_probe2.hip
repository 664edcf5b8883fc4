// Scale-lane map probe: A = B = 1.0 (e4m3 0x38), all scale words 0x7F7F7F7F (unit) except ONE lane
// of A whose word is given; prints the 16x16 C entries that differ from the unit result 128.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int OPSEL>
__global__ void probe(int lane_sel, int word, float* C) {
  const int l = threadIdx.x;
  i32x8 a, b;
  for (int w = 0; w < 8; ++w) a[w] = b[w] = 0x38383838;
  const int sa = l == lane_sel ? word : 0x7F7F7F7F;
  const int sb = 0x7F7F7F7F;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, OPSEL, sa, 0, sb);
  for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

int main() {
  float* dC;
  hipMalloc(&dC, 256 * 4);
  const int lanes[] = {0, 1, 5, 15, 16, 17, 31, 32, 47, 48, 63};
  const int words[] = {0x7F7F7F80, 0x7F7F807F, 0x7F807F7F, (int)0x807F7F7Fu};
  for (int opsel = 0; opsel < 2; ++opsel)
    for (int wi = 0; wi < 4; ++wi)
      for (int L : lanes) {
        if (opsel == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, L, words[wi], dC);
        else hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, L, words[wi], dC);
        float h[256];
        hipMemcpy(h, dC, sizeof h, hipMemcpyDeviceToHost);
        printf("opsel %d word %08x lane %2d:", opsel, words[wi], L);
        int n = 0;
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j)
            if (h[i * 16 + j] != 128.f) {
              if (n < 6) printf(" C[%d][%d]=%g", i, j, h[i * 16 + j]);
              ++n;
            }
        printf("  (%d entries differ; C[0][0]=%g)\n", n, h[0]);
      }
  return 0;
}
