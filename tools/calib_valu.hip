// Calibrates the SQ VALU lane counters on gfx950.  Run under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --kernel-trace
// and compare SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU per kernel:
//   lanes<64|32|8>   the same fma chain with 64, 32 and 8 active lanes
//   mix<K>           64 active lanes, one instruction class each:
//                    0 v_cmp + v_cndmask, 1 v_mul/v_sub with SGPR operands,
//                    2 packed fp32 (v_pk_mul/v_pk_add), 3 f64 fma, 4 v_rcp_f32
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int kLanes>
__global__ void __launch_bounds__(256) valu_lanes(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.5f;
  if (lane < kLanes) {
    for (int i = 0; i < iters; i++) {
      a = a * b + c;
      b = b * a + c;
      c = c * b + a;
      a = a * c + b;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a + b + c;
}

typedef float f2v __attribute__((ext_vector_type(2)));

template <int K>
__global__ void __launch_bounds__(256) valu_mix(float* out, int iters, float s0, float s1) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.5f;
  double da = a, db = b;
  f2v pa = {a, b}, pb = {b, c};
  for (int i = 0; i < iters; i++) {
    if constexpr (K == 0) {
      a = (a < b) ? a + c : b;
      b = (b > c) ? b : a;
      c = (c < a) ? a : c + b;
    } else if constexpr (K == 1) {
      a = a * s0 - s1;
      b = b * s1 - s0;
      c = c * s0 - a;
    } else if constexpr (K == 2) {
      pa = pa * pb + pa;
      pb = pb * pa + pb;
    } else if constexpr (K == 3) {
      da = da * db + 0.5;
      db = db * da + 0.25;
    } else {
      a = __builtin_amdgcn_rcpf(a + b);
      b = __builtin_amdgcn_rcpf(b + a);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a + b + c + (float)(da + db) + pa.x + pa.y + pb.x + pb.y;
}

int main(int argc, char** argv) {
  float* d = nullptr;
  const int blocks = 4096, iters = argc > 1 ? std::atoi(argv[1]) : 4096;
  if (hipMalloc(&d, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
  valu_lanes<64><<<blocks, 256>>>(d, iters);
  valu_lanes<32><<<blocks, 256>>>(d, iters);
  valu_lanes<8><<<blocks, 256>>>(d, iters);
  valu_mix<0><<<blocks, 256>>>(d, iters, 1.0001f, 0.5f);
  valu_mix<1><<<blocks, 256>>>(d, iters, 1.0001f, 0.5f);
  valu_mix<2><<<blocks, 256>>>(d, iters, 1.0001f, 0.5f);
  valu_mix<3><<<blocks, 256>>>(d, iters, 1.0001f, 0.5f);
  valu_mix<4><<<blocks, 256>>>(d, iters, 1.0001f, 0.5f);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("ok\n");
  return 0;
}
