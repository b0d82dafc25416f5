// VALU issue-rate calibration on gfx950: how many cycles does one SIMD spend
// per wave64 VALU instruction when several waves share it?  Each wave runs
// `iters` x (kChains independent fma chains x 8 unrolled), stamps s_memtime
// around its loop, and the host reports cycles per wave-instruction per SIMD
// (sum of instructions of the waves resident on a SIMD / elapsed cycles) and
// wall time via hipEvents.
//   usage: calib_issue [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int kChains, int kPacked>
__global__ void __launch_bounds__(256) fma_rate(float* out, unsigned long long* stamps, int iters) {
  float a[kChains];
#pragma unroll
  for (int c = 0; c < kChains; c++) a[c] = threadIdx.x * 1e-3f + c;
  const float b = 0.99999f, d = 1e-7f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if constexpr (kPacked) {
        typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int c = 0; c < kChains; c += 2) {
          f2 v = {a[c], a[c + 1]};
          f2 bb = {b, b}, dd = {d, d};
          asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(bb), "v"(dd));
          a[c] = v.x;
          a[c + 1] = v.y;
        }
      } else {
#pragma unroll
        for (int c = 0; c < kChains; c++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(d));
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kChains; c++) s += a[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    size_t w = blockIdx.x * 4 + threadIdx.x / 64;
    stamps[2 * w] = t0;
    stamps[2 * w + 1] = t1;
  }
}

// kMix 1: per chain v_fma + v_cmp + v_cndmask (compare/select, as in the quad tests);
// kMix 2: per chain v_fma + v_min + v_max3 (min/max trees); kMix 3: v_fma_f64
template <int kMix>
__global__ void __launch_bounds__(256) mix_rate(float* out, unsigned long long* stamps, int iters) {
  float a[8];
  double x[4];
#pragma unroll
  for (int c = 0; c < 8; c++) a[c] = threadIdx.x * 1e-3f + c;
#pragma unroll
  for (int c = 0; c < 4; c++) x[c] = a[c];
  const float b = 0.99999f, d = 1e-7f, lim = 0.5f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
#pragma unroll
      for (int c = 0; c < 8; c++) {
        if constexpr (kMix == 1) {
          asm volatile("v_fma_f32 %0, %0, %1, %2\n\tv_cmp_lt_f32 vcc, %0, %3\n\tv_cndmask_b32 %0, %0, %2, vcc"
                       : "+v"(a[c]) : "v"(b), "v"(d), "v"(lim) : "vcc");
        } else if constexpr (kMix == 2) {
          asm volatile("v_fma_f32 %0, %0, %1, %2\n\tv_min_f32 %0, %0, %1\n\tv_max3_f32 %0, %0, %2, %3"
                       : "+v"(a[c]) : "v"(b), "v"(d), "v"(lim));
        } else {
          if (c < 4) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"((double)b), "v"((double)d));
        }
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; c++) s += a[c];
#pragma unroll
  for (int c = 0; c < 4; c++) s += (float)x[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    size_t w = blockIdx.x * 4 + threadIdx.x / 64;
    stamps[2 * w] = t0;
    stamps[2 * w + 1] = t1;
  }
}

template <int kMix>
static void run_mix(const char* name, int blocks_per_cu, int iters, float* d, unsigned long long* st, int cus) {
  const int blocks = blocks_per_cu * cus;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  mix_rate<kMix><<<blocks, 256>>>(d, st, iters);
  hipEventRecord(e0);
  mix_rate<kMix><<<blocks, 256>>>(d, st, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)blocks * 4 * 2);
  hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  double cyc = 0;
  for (size_t w = 0; w < (size_t)blocks * 4; w++) cyc += double(h[2 * w + 1] - h[2 * w]);
  cyc /= blocks * 4.0;
  const double instr_per_wave = double(iters) * 8 * (kMix == 3 ? 4 : 24);
  const double clk = cyc / (ms * 1e-3);  // one wave spans ~the launch at 1 block/CU only
  std::printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"wave_cycles\": %.0f, "
              "\"wall_cpi_at_2.1GHz\": %.3f, \"wave_cpi\": %.3f, \"clk_est_GHz\": %.3f}\n",
              name, blocks_per_cu, ms, cyc, ms * 1e-3 * 2.1e9 / (instr_per_wave * blocks_per_cu),
              cyc / instr_per_wave, clk / 1e9);
}

template <int kChains, int kPacked>
static void run(const char* name, int blocks_per_cu, int iters, float* d, unsigned long long* st, int cus) {
  const int blocks = blocks_per_cu * cus;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  fma_rate<kChains, kPacked><<<blocks, 256>>>(d, st, iters);  // warm
  hipEventRecord(e0);
  fma_rate<kChains, kPacked><<<blocks, 256>>>(d, st, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)blocks * 4 * 2);
  hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  double cyc = 0;
  for (size_t w = 0; w < (size_t)blocks * 4; w++) cyc += double(h[2 * w + 1] - h[2 * w]);
  cyc /= blocks * 4.0;
  const double instr_per_wave = double(iters) * 8 * (kPacked ? kChains / 2 : kChains);
  const double waves_per_simd = blocks_per_cu;  // 4 waves per block, 4 SIMDs per CU
  // cycles the SIMD spends per wave-instruction, if the waves on it overlap fully
  const double cpi = cyc / (instr_per_wave * waves_per_simd);
  const double wall_cpi = ms * 1e-3 * 2.4e9 / (instr_per_wave * waves_per_simd);
  std::printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"chains\": %d, \"packed\": %d, \"ms\": %.4f, "
              "\"wave_cycles\": %.0f, \"simd_cycles_per_wave_instr\": %.3f, \"wall_cpi_at_2.4GHz\": %.3f}\n",
              name, blocks_per_cu, kChains, kPacked, ms, cyc, cpi, wall_cpi);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2048;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  float* d = nullptr;
  unsigned long long* st = nullptr;
  if (hipMalloc(&d, (size_t)8 * cus * 256 * 4) != hipSuccess) return 1;
  if (hipMalloc(&st, (size_t)8 * cus * 4 * 16) != hipSuccess) return 1;
  for (int w : {1, 2, 4, 5, 8}) run<8, 0>("fma8", w, iters, d, st, cus);
  for (int w : {1, 2, 4, 8}) run<1, 0>("fma1", w, iters, d, st, cus);
  for (int w : {1, 2, 4, 8}) run<8, 1>("pkfma8", w, iters, d, st, cus);
  for (int w : {1, 4, 5, 8}) run_mix<1>("fma_cmp_cnd", w, iters, d, st, cus);
  for (int w : {1, 4, 5, 8}) run_mix<2>("fma_min_max3", w, iters, d, st, cus);
  for (int w : {1, 4, 5, 8}) run_mix<3>("fma_f64", w, iters, d, st, cus);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  return 0;
}
