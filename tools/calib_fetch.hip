// Calibrates FETCH_SIZE / WRITE_SIZE on gfx950 for the render kernel's own
// access patterns, on known byte counts.  Run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace   (and a second pass with WRITE_SIZE)
// Kernels (one launch each, 2^28 lanes):
//   gather4   one random 4-B load per lane from a 16 GiB table (the RNG jump tables)
//   gather16  one random 16-B load per lane from a 16 GiB buffer (scattered history rows)
//   stream16  16-B loads, consecutive lanes -> consecutive 16 B (coalesced reference)
//   scatter16 one random 16-B store per lane into a 16 GiB buffer (history writes)
// The random index is a Wang hash of the lane id, so lines are almost never reused.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t hash(uint32_t s) {
  s = (s ^ 61u) ^ (s >> 16);
  s *= 9u;
  s = s ^ (s >> 4);
  s *= 0x27d4eb2du;
  return s ^ (s >> 15);
}

__global__ void gather4(const uint32_t* __restrict__ t, uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t v = t[hash(i)];  // 2^32 entries
  if (v == 0x12345678u) out[0] = i;
}
__global__ void gather16(const float4* __restrict__ t, uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const float4 v = t[hash(i) >> 2];  // 2^30 entries
  if (v.x == 1.2345f) out[0] = i;
}
__global__ void stream16(const float4* __restrict__ t, uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const float4 v = t[i];
  if (v.x == 1.2345f) out[0] = i;
}
__global__ void scatter16(float4* __restrict__ t) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  t[hash(i) >> 2] = make_float4(1.f, 2.f, 3.f, 0.f);
}

int main() {
  const size_t big = (size_t)16 << 30;
  const uint32_t lanes = 1u << 28;
  void* t = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&t, big) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(t, 0, big) != hipSuccess) return 2;
  const dim3 g(lanes / 256), b(256);
  gather4<<<g, b>>>(static_cast<const uint32_t*>(t), out);
  gather16<<<g, b>>>(static_cast<const float4*>(t), out);
  stream16<<<g, b>>>(static_cast<const float4*>(t), out);
  scatter16<<<g, b>>>(static_cast<float4*>(t));
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  std::printf("lanes %u: gather4 %.3e B, gather16/stream16/scatter16 %.3e B\n", lanes, 4.0 * lanes, 16.0 * lanes);
  return 0;
}
