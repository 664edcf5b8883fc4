// Which A-scale lane scales which (data lane, VGPR half)? A = 0 except lane X's VGPRs 4h..4h+3
// (16 bytes = 1.0), B = 1.0, scales unit except lane L of A (x2, opsel 0). C[0][0] = 16 or 32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(int X, int h, int L, float* C) {
  const int l = threadIdx.x;
  i32x8 a, b;
  for (int w = 0; w < 8; ++w) {
    a[w] = (l == X && (w >> 2) == h) ? 0x38383838 : 0;
    b[w] = 0x38383838;
  }
  const int sa = l == L ? 0x80 : 0x7F;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, 0x7F);
  for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

int main() {
  float* dC;
  (void)hipMalloc(&dC, 256 * 4);
  printf("data lane X, half h -> C[0][0] with the x2 scale on lane L = 0 / 16 / 32 / 48\n");
  for (int X = 0; X < 64; X += 16)
    for (int h = 0; h < 2; ++h) {
      printf("X=%2d h=%d:", X, h);
      for (int L = 0; L < 64; L += 16) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, X, h, L, dC);
        float c;
        (void)hipMemcpy(&c, dC, 4, hipMemcpyDeviceToHost);
        printf(" %5g", c);
      }
      printf("\n");
    }
  return 0;
}
