// trans_bias_bins -- mean signed error of v_exp_f32 / v_log_f32 / v_rcp_f32 per
// argument bin (diagnostic for the fast engine's flux bias).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k_eval(const float* __restrict__ x, float* __restrict__ out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = __builtin_amdgcn_exp2f(x[i]);
  out[n + i] = __builtin_amdgcn_logf(x[i] + 3.0f);  // log2 on [1, 5]
  out[2 * n + i] = __builtin_amdgcn_rcpf(x[i] + 3.0f);
}

int main() {
  const int per = 1 << 16, bins = 24;
  const int n = per * bins;
  std::vector<float> x(n);
  for (int b = 0; b < bins; ++b)
    for (int j = 0; j < per; ++j) x[b * per + j] = -3.0f + 0.25f * b + 0.25f * (j + 0.5f) / per;  // [-3, 3)
  float *dx, *dout;
  (void)hipMalloc(&dx, n * 4);
  (void)hipMalloc(&dout, 3 * n * 4);
  (void)hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  k_eval<<<(n + 255) / 256, 256>>>(dx, dout, n);
  std::vector<float> out(3 * n);
  (void)hipMemcpy(out.data(), dout, 3 * n * 4, hipMemcpyDeviceToHost);
  for (int f = 0; f < 3; ++f) {
    std::printf("%s:", f == 0 ? "exp2(x)" : f == 1 ? "log2(x+3)" : "rcp(x+3)");
    for (int b = 0; b < bins; ++b) {
      double s = 0;
      for (int j = 0; j < per; ++j) {
        const int i = b * per + j;
        const double a = f == 0 ? (double)x[i] : (double)(float)(x[i] + 3.0f);
        const double ref = f == 0 ? std::exp2(a) : f == 1 ? std::log2(a) : 1.0 / a;
        s += (out[f * n + i] - ref) / std::fabs(ref);
      }
      std::printf(" [%.2f]%+.1e", -3.0 + 0.25 * b, s / per);
    }
    std::printf("\n");
  }
  return 0;
}
