// exact-integer check of the assumed v_mfma_i32_32x32x32_i8 maps: lane l holds A[l&31][16(l>>5)+j] and
// B[16(l>>5)+j][l&31] (j = 0..15), D[row (r&3)+8(r>>2)+4(l>>5)][col l&31] in register r
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(const signed char* A, const signed char* B, int* D) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  signed char a[16], b[16];
  for (int j = 0; j < 16; ++j) { a[j] = A[r * 32 + 16 * h + j]; b[j] = B[(16 * h + j) * 32 + r]; }
  v4i av, bv; __builtin_memcpy(&av, a, 16); __builtin_memcpy(&bv, b, 16);
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int g = 0; g < 16; ++g) D[((g & 3) + 8 * (g >> 2) + 4 * h) * 32 + r] = c[g];
}
int main() {
  signed char hA[1024], hB[1024]; int hD[1024], ref[1024];
  srand(1);
  for (int i = 0; i < 1024; ++i) { hA[i] = (rand() % 15) - 7; hB[i] = (rand() % 255) - 127; }
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { int s = 0; for (int q = 0; q < 32; ++q) s += hA[i * 32 + q] * hB[q * 32 + j]; ref[i * 32 + j] = s; }
  signed char *dA, *dB; int* dD;
  if (hipMalloc(&dA, 1024) || hipMalloc(&dB, 1024) || hipMalloc(&dD, 4096)) return 2;
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 1024; ++i) bad += hD[i] != ref[i];
  printf("mfma_i32_32x32x32_i8 assumed maps: %d of 1024 wrong (D[0]=%d ref %d)\n", bad, hD[0], ref[0]);
  return bad != 0;
}
