// Probe: verify MFMA operand / accumulator lane maps on gfx950 with asymmetric integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// A: 32xK row-major, B: Kx32 row-major, K=2 ; D 32x32 row-major
__global__ void k32(const float* A, const float* B, float* D) {
  int l = threadIdx.x;
  float a = A[(l & 31) * 2 + (l >> 5)];
  float b = B[(l >> 5) * 32 + (l & 31)];
  f32x16 acc = {0};
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    int col = l & 31;
    D[row * 32 + col] = acc[r];
  }
}
// A: 16x4, B: 4x16
__global__ void k16(const float* A, const float* B, float* D) {
  int l = threadIdx.x;
  float a = A[(l & 15) * 4 + (l >> 4)];
  float b = B[(l >> 4) * 16 + (l & 15)];
  f32x4 acc = {0};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    int row = 4 * (l >> 4) + r;
    int col = l & 15;
    D[row * 16 + col] = acc[r];
  }
}
__global__ void k16d(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  f64x4 acc = {0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) + 4 * r;
    int col = l & 15;
    D[row * 16 + col] = acc[r];
  }
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// f16 32x32x16: A[i=l&31][k=8(l>>5)+j], B[k=8(l>>5)+j][j2=l&31] (as the bf16 map in the guide)
__global__ void k32h(const float* A, const float* B, float* D) {
  int l = threadIdx.x;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)A[(l & 31) * 16 + 8 * (l >> 5) + j];
    b[j] = (_Float16)B[(8 * (l >> 5) + j) * 32 + (l & 31)];
  }
  f32x16 acc = {0};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    D[row * 32 + (l & 31)] = acc[r];
  }
}
// f16 16x16x32: A[i=l&15][k=8(l>>4)+j], B[k=8(l>>4)+j][l&15]; D row=4(l>>4)+r
__global__ void k16h(const float* A, const float* B, float* D) {
  int l = threadIdx.x;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)A[(l & 15) * 32 + 8 * (l >> 4) + j];
    b[j] = (_Float16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f32x4 acc = {0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

template <typename T>
int check(const T* A, const T* B, const T* D, int M, int N, int K, const char* name) {
  int bad = 0;
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      double s = 0;
      for (int k = 0; k < K; ++k) s += (double)A[i * K + k] * (double)B[k * N + j];
      if (fabs(s - (double)D[i * N + j]) > 1e-9) ++bad;
    }
  printf("%s: %d mismatches of %d\n", name, bad, M * N);
  return bad;
}

int main() {
  int bad = 0;
  {
    float hA[64], hB[64], hD[1024];
    for (int i = 0; i < 64; ++i) { hA[i] = (float)(i * 3 + 1); hB[i] = (float)((i * 7) % 13 - 5); }
    float *dA, *dB, *dD;
    hipMalloc(&dA, 256); hipMalloc(&dB, 256); hipMalloc(&dD, 4096);
    hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
    k32<<<1, 64>>>(dA, dB, dD);
    hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
    bad += check(hA, hB, hD, 32, 32, 2, "f32_32x32x2");
    k16<<<1, 64>>>(dA, dB, dD);
    hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    bad += check(hA, hB, hD, 16, 16, 4, "f32_16x16x4");
  }
  {
    double hA[64], hB[64], hD[256];
    for (int i = 0; i < 64; ++i) { hA[i] = (double)(i * 3 + 1); hB[i] = (double)((i * 7) % 13 - 5); }
    double *dA, *dB, *dD;
    hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048);
    hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
    k16d<<<1, 64>>>(dA, dB, dD);
    hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
    bad += check(hA, hB, hD, 16, 16, 4, "f64_16x16x4");
  }
  {
    float hA[512], hB[512], hD[1024];
    for (int i = 0; i < 512; ++i) { hA[i] = (float)((i * 5) % 17 - 8); hB[i] = (float)((i * 7) % 13 - 5); }
    float *dA, *dB, *dD;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dD, 4096);
    hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    k32h<<<1, 64>>>(dA, dB, dD);
    hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
    bad += check(hA, hB, hD, 32, 32, 16, "f16_32x32x16");
    k16h<<<1, 64>>>(dA, dB, dD);
    hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    bad += check(hA, hB, hD, 16, 16, 32, "f16_16x16x32");
  }
  printf("TOTAL_BAD=%d\n", bad);
  return bad ? 1 : 0;
}
