// trans_bias -- signed error of the gfx950 fp32 transcendental instructions
// (v_rcp_f32, v_log_f32, v_exp_f32, v_sqrt_f32) against fp64 references,
// over the argument ranges the fast engine feeds them.  Mean relative error =
// bias; it accumulates in the state through the energy fluxes.
//   hipcc --offload-arch=gfx950 -O3 -o tools/trans_bias tools/trans_bias.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void k_eval(const float* __restrict__ x, float* __restrict__ out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  out[0 * n + i] = __builtin_amdgcn_rcpf(v);
  out[1 * n + i] = __builtin_amdgcn_logf(v);    // log2
  out[2 * n + i] = __builtin_amdgcn_exp2f(v * 0.01f - 5.0f);  // exp2 on [-5, 5]
  out[3 * n + i] = __builtin_sqrtf(v);
  // Newton-refined reciprocal: r + r*(1 - v*r)
  const float r = __builtin_amdgcn_rcpf(v);
  out[4 * n + i] = fmaf(r, fmaf(-v, r, 1.0f), r);
}

int main() {
  const int n = 1 << 22;
  std::vector<float> x(n);
  std::mt19937 rng(7);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (int i = 0; i < n; ++i) x[i] = (float)std::exp2(u(rng) * 10.0);  // [2^-10, 2^10]
  float *dx, *dout;
  (void)hipMalloc(&dx, n * 4);
  (void)hipMalloc(&dout, 5 * n * 4);
  (void)hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  k_eval<<<(n + 255) / 256, 256>>>(dx, dout, n);
  std::vector<float> out(5 * n);
  (void)hipMemcpy(out.data(), dout, 5 * n * 4, hipMemcpyDeviceToHost);
  const char* names[5] = {"v_rcp_f32", "v_log_f32 (log2)", "v_exp_f32 (exp2)", "sqrt", "rcp + 1 Newton step"};
  for (int f = 0; f < 5; ++f) {
    double s = 0, mx = 0, su = 0;
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
      const double xv = x[i];
      double ref;
      switch (f) {
        case 0: case 4: ref = 1.0 / xv; break;
        case 1: ref = std::log2(xv); break;
        case 2: ref = std::exp2((double)(float)(x[i] * 0.01f - 5.0f)); break;
        default: ref = std::sqrt(xv); break;
      }
      if (f == 1 && std::fabs(ref) < 1e-3) continue;
      const double g = out[f * n + i];
      const double rel = (g - ref) / std::fabs(ref);
      const double ulp = std::ldexp(1.0, std::ilogb(ref) - 23);
      s += rel; mx = std::fmax(mx, std::fabs(rel)); su += (g - ref) / ulp; ++cnt;
    }
    std::printf("{\"fn\": \"%s\", \"mean_rel\": %.3e, \"max_rel\": %.3e, \"mean_ulp\": %+.3f}\n", names[f], s / cnt, mx, su / cnt);
  }
  return 0;
}
