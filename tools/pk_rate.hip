// pk_rate -- VALU issue rate of packed fp32 (v_pk_fma_f32, two lanes' worth
// per instruction) against scalar fp32 (v_fma_f32) and fp64 (v_fma_f64) on
// gfx950: the question of VERDICT r5 item 3 (two cells per lane with packed
// FP32 flux arithmetic).  Each thread runs 8 independent FMA chains of 4096
// steps; the packed kernel does the same number of multiply-adds in half as
// many instructions.  Prints FMA/s and instructions/s for each.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pk_rate tools/pk_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_f32(float* out, float a, float b) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3f + j;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(a), "v"(b));  // no SLP packing
  }
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk(float* out, float a, float b) {
  float2v x[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] = float2v{threadIdx.x * 1e-3f + 2 * j, threadIdx.x * 1e-3f + 2 * j + 1};
  const float2v av = {a, a}, bv = {b, b};
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(av), "v"(bv));
  }
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += x[j].x + x[j].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_f64(double* out, double a, double b) {
  double x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3 + j;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[j]) : "v"(a), "v"(b));
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus * 16, threads = 256;  // 16 workgroups of 4 waves per CU: 16 waves per SIMD queued
  const double n_thr = (double)blocks * threads;
  float* o32;
  double* o64;
  (void)hipMalloc(&o32, (size_t)blocks * threads * 4);
  (void)hipMalloc(&o64, (size_t)blocks * threads * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[3] = {"v_fma_f32 (scalar fp32)", "v_pk_fma_f32 (packed fp32)", "v_fma_f64"};
  for (int rep = 0; rep < 3; ++rep) {
    for (int k = 0; k < 3; ++k) {
      (void)hipEventRecord(e0);
      if (k == 0) k_f32<<<blocks, threads>>>(o32, 0.999f, 1e-3f);
      if (k == 1) k_pk<<<blocks, threads>>>(o32, 0.999f, 1e-3f);
      if (k == 2) k_f64<<<blocks, threads>>>(o64, 0.999, 1e-3);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double fmas = n_thr * kIters * 8.0;
      const double insts = fmas / (k == 1 ? 2.0 : 1.0) / 64.0;  // wave instructions
      if (rep == 2)
        printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"fma_per_s\": %.4g, \"wave_insts_per_s\": %.4g, "
               "\"cycles_per_wave_inst_per_simd_at_2.4GHz\": %.3f}\n",
               names[k], ms, fmas / (ms * 1e-3), insts / (ms * 1e-3), (4.0 * cus * 2.4e9) / (insts / (ms * 1e-3)));
    }
  }
  return 0;
}
