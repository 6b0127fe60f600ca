// Issue cost of the VALU instruction classes the pipeline's kernels execute, on a
// full chip (8 waves per SIMD, every CU busy): each kernel runs kIter rounds of
// 8 independent chains of one operation per lane; cycles per wave64 instruction
// per SIMD = kernel time x clock x SIMDs / (waves x instructions per wave).
// The clock is read in the kernel (s_memtime ticks vs the wall clock of
// s_memrealtime, 100 MHz) so DVFS does not bias the result.
// Output: one JSON line per class.  (tools/ only: DESIGN.md section 5's issue
// ceiling weights the per-class VALU counters of profiles/ by these costs.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIter = 4096;
constexpr int kChains = 8;

#define OPK(name, T, init, expr)                                                      \
  __global__ __launch_bounds__(256) void name(T* out, uint64_t* clk, T seed) {        \
    T a[kChains];                                                                     \
    for (int i = 0; i < kChains; i++) a[i] = seed + (T)(threadIdx.x + i) * (T)init;   \
    uint64_t c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime(); \
    for (int it = 0; it < kIter; it++) {                                              \
      _Pragma("unroll") for (int i = 0; i < kChains; i++) { T x = a[i]; a[i] = expr; } \
    }                                                                                 \
    uint64_t c1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime(); \
    T s = 0;                                                                          \
    for (int i = 0; i < kChains; i++) s += a[i];                                      \
    out[blockIdx.x * 256 + threadIdx.x] = s;                                          \
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = c1 - c0; clk[1] = r1 - r0; }  \
  }

OPK(k_add_f32, float, 1e-3f, x + 1.0001f)
OPK(k_fma_f32, float, 1e-3f, x * 0.9999f + 1e-4f)
OPK(k_fma_f64, double, 1e-3, x * 0.9999 + 1e-4)
OPK(k_add_f64, double, 1e-3, x + 1.0001)
OPK(k_sqrt_f32, float, 1e-3f, __builtin_amdgcn_sqrtf(x) + 1.0f)
OPK(k_rcp_f32, float, 1e-3f, __builtin_amdgcn_rcpf(x) + 1.0f)
OPK(k_rcp_f64, double, 1e-3, __builtin_amdgcn_rcp(x) + 1.0)
OPK(k_sqrt_f64, double, 1e-3, __builtin_amdgcn_sqrt(x) + 1.0)
OPK(k_mul_u32, uint32_t, 3u, x * 2654435761u + 1u)
OPK(k_add_u64, uint64_t, 3ull, x + 0x9e3779b97f4a7c15ull)
OPK(k_cvt_f64_f32, double, 1e-3, (double)(float)x + 1.0)

template <typename T>
static void run(const char* name, void (*k)(T*, uint64_t*, T), int ncu, const char* note) {
  const int blocks = ncu * 8;  // 256-thread blocks: 4 waves each, 8 per CU = 8 waves per SIMD
  T* out;
  uint64_t* clk;
  hipMalloc(&out, sizeof(T) * blocks * 256);
  hipMalloc(&clk, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, (T)1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, (T)1);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  uint64_t h[2];
  hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = h[1] ? (double)h[0] / ((double)h[1] * 10.0) : 0.0;  // s_memrealtime: 100 MHz
  const double waves = (double)blocks * 4, instr = (double)kIter * kChains;
  const double cyc = (ms / reps) * 1e-3 * ghz * 1e9 * (ncu * 4) / (waves * instr);
  std::printf("{\"class\":\"%s\",\"ms\":%.4f,\"clock_ghz\":%.3f,\"cycles_per_wave_instr_per_simd\":%.3f,\"note\":\"%s\"}\n",
              name, ms / reps, ghz, cyc, note);
  hipFree(out);
  hipFree(clk);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  run<float>("add_f32", k_add_f32, ncu, "v_add_f32");
  run<float>("fma_f32", k_fma_f32, ncu, "v_fma_f32 / v_fmac_f32");
  run<double>("fma_f64", k_fma_f64, ncu, "v_fma_f64");
  run<double>("add_f64", k_add_f64, ncu, "v_add_f64");
  run<float>("sqrt_f32", k_sqrt_f32, ncu, "v_sqrt_f32 + v_add_f32");
  run<float>("rcp_f32", k_rcp_f32, ncu, "v_rcp_f32 + v_add_f32");
  run<double>("rcp_f64", k_rcp_f64, ncu, "v_rcp_f64 + v_add_f64");
  run<double>("sqrt_f64", k_sqrt_f64, ncu, "v_sqrt_f64 + v_add_f64");
  run<uint32_t>("mul_u32", k_mul_u32, ncu, "v_mul_lo_u32 + v_add_u32");
  run<uint64_t>("add_u64", k_add_u64, ncu, "v_add_co_u32 + v_addc_co_u32");
  run<double>("cvt_f64_f32", k_cvt_f64_f32, ncu, "v_cvt_f32_f64 + v_cvt_f64_f32 + v_add_f64");
  return 0;
}
