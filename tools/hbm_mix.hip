// hbm_mix -- HBM bandwidth ceiling for the fused kernel's access mix on MI355X.
//
// Streams `cells` fp32 elements per plane: each "step" a thread reads R planes
// and writes W planes at its cell (coalesced, 4 B per lane per plane), the
// k_fused pattern (R = 6: five forcing fields + window slot; W = 7: window slot
// + six outputs).  Reports GB/s for several (R, W) mixes so the measured
// k_fused rate can be placed against what this read/write mix can reach.
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_mix tools/hbm_mix.hip
//   tools/hbm_mix [cells=67108864] [steps=24] [workgroups=2048] [skew=0] [il|pf|tb|cal]
// skew: extra cells between consecutive planes (plane stride = cells + skew),
// to test whether power-of-two plane strides cost HBM channel balance.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

template <int V> struct Vec;
template <> struct Vec<1> { using T = float; };
template <> struct Vec<2> { using T = float2; };
template <> struct Vec<4> { using T = float4; };
__device__ __forceinline__ float hsum(float v) { return v; }
__device__ __forceinline__ float hsum(float2 v) { return v.x + v.y; }
__device__ __forceinline__ float hsum(float4 v) { return v.x + v.y + v.z + v.w; }
__device__ __forceinline__ void splat(float& o, float a) { o = a; }
__device__ __forceinline__ void splat(float2& o, float a) { o = make_float2(a, a + 1.0f); }
__device__ __forceinline__ void splat(float4& o, float a) { o = make_float4(a, a + 1.0f, a + 2.0f, a + 3.0f); }

// Store cache policy of the 4-byte stores (POL > 0, V = 1): the gfx950
// global_store_dword bits, written out in asm (the compiler emits only plain and nt).
template <int POL>
__device__ __forceinline__ void store_pol(float* p, float v) {
  if constexpr (POL == 1) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 2) asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 3) asm volatile("global_store_dword %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 4) asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 5) asm volatile("global_store_dword %0, %1, off sc0 nt" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 6) asm volatile("global_store_dword %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
}

// V floats (V adjacent cells) per lane per plane; NT: non-temporal stores;
// POL: a store cache policy of store_pol instead
template <int R, int W, int V, bool NT = false, int POL = 0>
__global__ __launch_bounds__(256) void k_mix(const float* __restrict__ in, float* __restrict__ out, uint32_t n,
                                             int steps, int frames, uint32_t ps) {
  using T = typename Vec<V>::T;
  const uint32_t nv = n / V;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float acc = 0.0f;
    for (int s = 0; s < steps; ++s) {
      const float* fin = in + (size_t)(s % frames) * R * ps;
      T v[R > 0 ? R : 1];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = reinterpret_cast<const T*>(fin + (size_t)r * ps)[i];
#pragma unroll
      for (int r = 0; r < R; ++r) acc += hsum(v[r]);
      float* fo = out + (size_t)(s % frames) * W * ps;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        T o;
        splat(o, acc + (float)w);
        T* dst = reinterpret_cast<T*>(fo + (size_t)w * ps) + i;
        if constexpr (POL > 0) { static_assert(V == 1, "policy stores are 4 B"); store_pol<POL>((float*)dst, hsum(o)); }
        else if constexpr (NT && V == 2)  // 8-byte lanes: the nontemporal builtin takes no float2
          __builtin_nontemporal_store(*reinterpret_cast<const unsigned long long*>(&o),
                                      reinterpret_cast<unsigned long long*>(dst));
        else if constexpr (NT) __builtin_nontemporal_store(o, dst);
        else *dst = o;
      }
    }
    if (W == 0 && acc == -1.0f) out[i] = acc;  // keep the reads alive
  }
}

// Block-interleaved layout: within a frame, cell i of plane r sits at
// ((i / IL) * P + r) * IL + i % IL (P planes), so one wave's P accesses of a
// step fall in one contiguous P*IL*4-byte run instead of P separate planes.
template <int R, int W, int IL>
__global__ __launch_bounds__(256) void k_mix_il(const float* __restrict__ in, float* __restrict__ out, uint32_t n,
                                                int steps, int frames) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t blk = i / IL, off = i % IL;
    float acc = 0.0f;
    for (int s = 0; s < steps; ++s) {
      const float* fin = in + (size_t)(s % frames) * R * n + (size_t)blk * R * IL + off;
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = fin[r * IL];
#pragma unroll
      for (int r = 0; r < R; ++r) acc += v[r];
      float* fo = out + (size_t)(s % frames) * W * n + (size_t)blk * W * IL + off;
#pragma unroll
      for (int w = 0; w < W; ++w) fo[w * IL] = acc + (float)w;
    }
  }
}

static int g_blocks = 256 * 8;
static uint32_t g_skew = 0;

template <int R, int W, int V = 1, bool NT = false, int POL = 0>
void run(const char* name, float* in, float* out, uint32_t n, int steps, int frames) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int blocks = g_blocks;
  const uint32_t ps = n + g_skew;
  k_mix<R, W, V, NT, POL><<<blocks, 256>>>(in, out, n, steps, frames, ps);  // warm-up
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(a));
    k_mix<R, W, V, NT, POL><<<blocks, 256>>>(in, out, n, steps, frames, ps);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double bytes = (double)n * steps * 4.0 * (R + W);
  std::printf("{\"mix\": \"%s\", \"read_planes\": %d, \"write_planes\": %d, \"bytes_per_lane\": %d, \"blocks\": %d, \"skew\": %u, \"GBps\": %.1f, \"ms\": %.3f}\n",
              name, R, W, 4 * V, g_blocks, g_skew, bytes / (best * 1e-3) / 1e9, best);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

template <int R, int W, int IL>
void run_il(const char* name, float* in, float* out, uint32_t n, int steps, int frames) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  k_mix_il<R, W, IL><<<g_blocks, 256>>>(in, out, n, steps, frames);  // warm-up
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(a));
    k_mix_il<R, W, IL><<<g_blocks, 256>>>(in, out, n, steps, frames);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double bytes = (double)n * steps * 4.0 * (R + W);
  std::printf("{\"mix\": \"%s\", \"read_planes\": %d, \"write_planes\": %d, \"interleave_cells\": %d, \"blocks\": %d, \"GBps\": %.1f, \"ms\": %.3f}\n",
              name, R, W, IL, g_blocks, bytes / (best * 1e-3) / 1e9, best);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}


// Software-pipelined variant: each thread keeps D steps of reads in flight
// (register ring, loads of step s+D issued before step s is consumed), the
// k_fused structure with a deeper read-ahead.  Requires steps % D == 0.
template <int R, int W, int D, int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_mix_pf(const float* __restrict__ in, float* __restrict__ out,
                                                       uint32_t n, int steps, int frames) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float buf[D][R > 0 ? R : 1];
    auto fetch = [&](int s, float (&b)[R > 0 ? R : 1]) {
      const int ss = s < steps ? s : steps - 1;
      const float* fin = in + (size_t)(ss % frames) * R * n + i;
#pragma unroll
      for (int r = 0; r < R; ++r) b[r] = __builtin_nontemporal_load(fin + (size_t)r * n);
    };
#pragma unroll
    for (int j = 0; j < D; ++j) fetch(j, buf[j]);
    float acc = 0.0f;
    for (int s0 = 0; s0 < steps; s0 += D) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int r = 0; r < R; ++r) acc += buf[j][r];
        fetch(s0 + j + D, buf[j]);
        float* fo = out + (size_t)((s0 + j) % frames) * W * n + i;
#pragma unroll
        for (int w = 0; w < W; ++w) __builtin_nontemporal_store(acc + (float)w, fo + (size_t)w * n);
      }
    }
    if (W == 0 && acc == -1.0f) out[i] = acc;  // keep the reads alive
  }
}

template <int R, int W, int D, int WAVES>
void run_pf(const char* name, float* in, float* out, uint32_t n, int steps, int frames) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  k_mix_pf<R, W, D, WAVES><<<g_blocks, 256>>>(in, out, n, steps, frames);  // warm-up
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(a));
    k_mix_pf<R, W, D, WAVES><<<g_blocks, 256>>>(in, out, n, steps, frames);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double bytes = (double)n * steps * 4.0 * (R + W);
  std::printf("{\"mix\": \"%s\", \"read_planes\": %d, \"write_planes\": %d, \"prefetch_steps\": %d, \"min_waves_per_simd\": %d, \"blocks\": %d, \"GBps\": %.1f, \"ms\": %.3f}\n",
              name, R, W, D, WAVES, g_blocks, bytes / (best * 1e-3) / 1e9, best);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}


// Time-blocked output layout: the W planes a step writes for a block of IL
// cells sit next to that block's previous steps, i.e. out[(blk*steps + s)*W*IL
// + w*IL + off]; reads stay planar.  A workgroup's writes over its steps then
// fill one contiguous region instead of W planes x steps scattered regions.
template <int R, int W, int IL>
__global__ __launch_bounds__(256) void k_mix_tb(const float* __restrict__ in, float* __restrict__ out, uint32_t n,
                                                int steps, int frames) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t blk = i / IL, off = i % IL;
    float acc = 0.0f;
    for (int s = 0; s < steps; ++s) {
      const float* fin = in + (size_t)(s % frames) * R * n + i;
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = fin[(size_t)r * n];
#pragma unroll
      for (int r = 0; r < R; ++r) acc += v[r];
      float* fo = out + ((size_t)blk * steps + s) * W * IL + off;
#pragma unroll
      for (int w = 0; w < W; ++w) __builtin_nontemporal_store(acc + (float)w, fo + (size_t)w * IL);
    }
  }
}

template <int R, int W, int IL>
void run_tb(const char* name, float* in, float* out, uint32_t n, int steps, int frames) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  k_mix_tb<R, W, IL><<<g_blocks, 256>>>(in, out, n, steps, frames);  // warm-up
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(a));
    k_mix_tb<R, W, IL><<<g_blocks, 256>>>(in, out, n, steps, frames);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double bytes = (double)n * steps * 4.0 * (R + W);
  std::printf("{\"mix\": \"%s\", \"read_planes\": %d, \"write_planes\": %d, \"time_block_cells\": %d, \"blocks\": %d, \"GBps\": %.1f, \"ms\": %.3f}\n",
              name, R, W, IL, g_blocks, bytes / (best * 1e-3) / 1e9, best);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)std::strtoul(argv[1], nullptr, 10) : 67108864u;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 24;
  if (argc > 3) g_blocks = std::atoi(argv[3]);
  if (argc > 4) g_skew = (uint32_t)std::strtoul(argv[4], nullptr, 10);
  if (g_skew % 4) { std::fprintf(stderr, "skew must be a multiple of 4 cells\n"); return 1; }
  const int frames = steps;  // one distinct frame per step, as k_fused (no address is touched twice)
  float *in, *out;
  CHECK(hipMalloc(&in, (size_t)(n + g_skew) * 4 * 7 * frames));
  CHECK(hipMalloc(&out, (size_t)(n + g_skew) * 4 * 7 * frames));
  CHECK(hipMemset(in, 0, (size_t)(n + g_skew) * 4 * 7 * frames));
  CHECK(hipMemset(out, 0, (size_t)(n + g_skew) * 4 * 7 * frames));
  if (argc > 5 && std::string(argv[5]) == "tb") {  // time-blocked output layout experiment only
    run<6, 7, 1, true>("k_fused step mix, planar, nt stores", in, out, n, steps, frames);
    run_tb<6, 7, 256>("k_fused step mix, time-blocked outputs (256 cells)", in, out, n, steps, frames);
    run_tb<6, 7, 1024>("k_fused step mix, time-blocked outputs (1024 cells)", in, out, n, steps, frames);
    run<6, 7, 1, true>("k_fused step mix, planar, nt stores", in, out, n, steps, frames);
    run_tb<6, 7, 256>("k_fused step mix, time-blocked outputs (256 cells)", in, out, n, steps, frames);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
  }
  if (argc > 5 && std::string(argv[5]) == "pf") {  // read-ahead depth experiment only
    run<6, 7, 1, true>("k_fused step mix, plain loop, nt stores", in, out, n, steps, frames);
    run_pf<6, 7, 1, 4>("k_fused step mix, read-ahead 1", in, out, n, steps, frames);
    run_pf<6, 7, 2, 4>("k_fused step mix, read-ahead 2", in, out, n, steps, frames);
    run_pf<6, 7, 4, 4>("k_fused step mix, read-ahead 4", in, out, n, steps, frames);
    run_pf<6, 7, 4, 2>("k_fused step mix, read-ahead 4, 2 waves/SIMD bound", in, out, n, steps, frames);
    run_pf<6, 7, 8, 2>("k_fused step mix, read-ahead 8, 2 waves/SIMD bound", in, out, n, steps, frames);
    run_pf<7, 0, 1, 4>("read only, read-ahead 1", in, out, n, steps, frames);
    run_pf<7, 0, 4, 4>("read only, read-ahead 4", in, out, n, steps, frames);
    run_pf<1, 1, 4, 4>("copy, read-ahead 4", in, out, n, steps, frames);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
  }
  if (argc > 5 && std::string(argv[5]) == "il") {  // layout experiment only
    run<6, 7>("k_fused step mix (6 read, 7 write), planar", in, out, n, steps, frames);
    run_il<6, 7, 64>("k_fused step mix, 64-cell block interleave", in, out, n, steps, frames);
    run_il<6, 7, 256>("k_fused step mix, 256-cell block interleave", in, out, n, steps, frames);
    run_il<6, 7, 1024>("k_fused step mix, 1024-cell block interleave", in, out, n, steps, frames);
    run<6, 7>("k_fused step mix (6 read, 7 write), planar", in, out, n, steps, frames);
    run_il<6, 7, 64>("k_fused step mix, 64-cell block interleave", in, out, n, steps, frames);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
  }
  if (argc > 5 && std::string(argv[5]) == "pol") {  // store cache-policy experiment only
    for (int rep = 0; rep < 2; ++rep) {
      run<6, 7, 1, false>("k_fused step mix, plain stores", in, out, n, steps, frames);
      run<6, 7, 1, true>("k_fused step mix, nt stores", in, out, n, steps, frames);
      run<6, 7, 1, false, 1>("k_fused step mix, sc1 stores", in, out, n, steps, frames);
      run<6, 7, 1, false, 2>("k_fused step mix, sc0 sc1 stores", in, out, n, steps, frames);
      run<6, 7, 1, false, 3>("k_fused step mix, sc1 nt stores", in, out, n, steps, frames);
      run<6, 7, 1, false, 4>("k_fused step mix, sc0 sc1 nt stores", in, out, n, steps, frames);
      run<6, 7, 1, false, 5>("k_fused step mix, sc0 nt stores", in, out, n, steps, frames);
      run<6, 7, 1, false, 6>("k_fused step mix, sc0 stores", in, out, n, steps, frames);
    }
    run<0, 7, 1, true>("write only, nt stores", in, out, n, steps, frames);
    run<0, 7, 1, false, 1>("write only, sc1 stores", in, out, n, steps, frames);
    run<0, 7, 1, false, 4>("write only, sc0 sc1 nt stores", in, out, n, steps, frames);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
  }
  if (argc > 5 && std::string(argv[5]) == "cal") {  // PMC calibration: known bytes per dispatch
    // rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) -- tools/hbm_mix <n> <steps> <blocks> 0 cal:
    // each kernel instance moves exactly n*steps*4*(R or W) bytes per dispatch, so
    // the counter / byte ratio calibrates the gfx950 correction for 4 B lanes
    // (k_fused's width) against 16 B lanes (the guide's calibration).
    run<7, 0>("cal read only 4 B/lane", in, out, n, steps, frames);
    run<7, 0, 4>("cal read only 16 B/lane", in, out, n, steps, frames);
    run<7, 0, 2>("cal read only 8 B/lane", in, out, n, steps, frames);  // the fp64 engine's width
    run<0, 7, 2, true>("cal write only 8 B/lane nt", in, out, n, steps, frames);
    run<0, 7>("cal write only 4 B/lane", in, out, n, steps, frames);
    run<0, 7, 1, true>("cal write only 4 B/lane nt", in, out, n, steps, frames);
    run<6, 7, 1, true>("cal k_fused mix 4 B/lane nt", in, out, n, steps, frames);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
  }
  run<6, 7>("k_fused step mix (6 read, 7 write)", in, out, n, steps, frames);
  run<6, 7, 1, true>("k_fused step mix, non-temporal stores", in, out, n, steps, frames);
  run<7, 0>("read only (7 planes)", in, out, n, steps, frames);
  run<0, 7>("write only (7 planes)", in, out, n, steps, frames);
  run<1, 1>("copy (1 read, 1 write)", in, out, n, steps, frames);
  run<6, 1>("read-heavy (6 read, 1 write)", in, out, n, steps, frames);
  run<6, 7, 2>("k_fused step mix, 8 B/lane", in, out, n, steps, frames);
  run<6, 7, 4>("k_fused step mix, 16 B/lane", in, out, n, steps, frames);
  run<7, 0, 4>("read only, 16 B/lane", in, out, n, steps, frames);
  run<0, 7, 4>("write only, 16 B/lane", in, out, n, steps, frames);
  run<1, 1, 4>("copy, 16 B/lane", in, out, n, steps, frames);
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  return 0;
}
