// Probe: lane/k layout of v_mfma_i32_16x16x64_i8 on gfx950 and zero-copy host-mapped I/O.
// Hypothesis (symmetric A/B): lane l holds A[row l&15][k = 16*(l>>4) + s], s = byte 0..15,
// B[k = 16*(l>>4) + s][col l&15]; C/D: col = l&15, row = 4*(l>>4) + i.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const signed char* A, const signed char* B, int* C) {
  int l = threadIdx.x;
  v4i a, b;
  __builtin_memcpy(&a, A + l * 16, 16);
  __builtin_memcpy(&b, B + l * 16, 16);
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[l * 4 + i] = c[i];
}
__global__ void zc(const unsigned char* in, unsigned char* out, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = in[i] ^ 0x5a;
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
  int n = 0; CK(hipGetDeviceCount(&n)); printf("devices=%d\n", n);
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0)); printf("name=%s arch=%s cus=%d lds=%zu\n", p.name, p.gcnArchName, p.multiProcessorCount, p.sharedMemPerBlock);
  signed char hA[16][64], hB[64][16];
  srand(7);
  for (int r = 0; r < 16; ++r) for (int k = 0; k < 64; ++k) hA[r][k] = (signed char)(rand() % 19 - 9);
  for (int k = 0; k < 64; ++k) for (int c = 0; c < 16; ++c) hB[k][c] = (signed char)(rand() % 23 - 11);
  signed char la[64 * 16], lb[64 * 16];
  for (int l = 0; l < 64; ++l) for (int s = 0; s < 16; ++s) {
    int k = 16 * (l >> 4) + s;
    la[l * 16 + s] = hA[l & 15][k];
    lb[l * 16 + s] = hB[k][l & 15];
  }
  signed char *dA, *dB; int* dC;
  CK(hipMalloc(&dA, 1024)); CK(hipMalloc(&dB, 1024)); CK(hipMalloc(&dC, 64 * 4 * 4));
  CK(hipMemcpy(dA, la, 1024, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, lb, 1024, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  int hc[256]; CK(hipMemcpy(hc, dC, 1024, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int i = 0; i < 4; ++i) {
    int row = 4 * (l >> 4) + i, col = l & 15, ref = 0;
    for (int k = 0; k < 64; ++k) ref += hA[row][k] * hB[k][col];
    if (ref != hc[l * 4 + i]) ++bad;
  }
  printf("mfma_i32_16x16x64_i8 layout hypothesis: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
  unsigned char *hin, *hout, *din, *dout;
  CK(hipHostMalloc((void**)&hin, 4096, hipHostMallocMapped)); CK(hipHostMalloc((void**)&hout, 4096, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&din, hin, 0)); CK(hipHostGetDevicePointer((void**)&dout, hout, 0));
  for (int i = 0; i < 4096; ++i) hin[i] = (unsigned char)i;
  hipLaunchKernelGGL(zc, dim3(1), dim3(256), 0, 0, din, dout, 4096);
  CK(hipDeviceSynchronize());
  int zbad = 0; for (int i = 0; i < 4096; ++i) zbad += hout[i] != (unsigned char)(i ^ 0x5a);
  printf("zero-copy host-mapped: %s (same_ptr=%d)\n", zbad ? "FAIL" : "PASS", (int)(din == hin));
  return bad || zbad;
}
