// rtp_bvh_gpu.hip -- device-side sphere BVH build (the
// role of VTK-m's LinearBVH behind SphereIntersector::SetData, reference
// SphereIntersector.cxx:46-76 / AABBSurface.h), for scenes too large for the
// host's binned-SAH build in rtp_host.cpp.
//
// Linear BVH (Karras 2012) over the sphere centres:
//   1. 30-bit Morton code of each centre in the centres' bounding box;
//   2. sort (code, sphere) pairs with rocPRIM's radix sort (hipCUB);
//   3. one thread per internal node finds its key range and split (duplicate
//      codes are split by position), recording children and parents;
//   4. bottom-up boxes and subtree sizes (one thread per leaf climbs; the
//      second arrival at a node merges its children);
//   5. flatten: for each of the 8 ray-direction octants, each node finds its
//      depth-first position by climbing to the root (near child first on the
//      node's split axis: the axis of the Morton bit that splits it), and is
//      written as a threaded node (skip = position + subtree size).
// The output is exactly the layout the render kernels walk (rtp_layout.hpp
// BvhNode, 8 octant copies, one-sphere leaves embedding the sphere), so a
// tree from either builder is traversed by the same code.  The closest hit is
// the (t, sphere index) minimum in both cases, so renders are bit-identical
// whichever tree is used (tests/test_gpu_bvh.py).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "rtp_layout.hpp"

namespace rtp {
namespace {

// spread the low 10 bits of v to every third bit
__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ void k_morton(const float4* __restrict__ cr, int n, float3 lo, float3 inv_ext, uint32_t* __restrict__ code,
                         uint32_t* __restrict__ idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 s = cr[i];
  auto q = [](float v) { return (uint32_t)fminf(fmaxf(v * 1024.0f, 0.0f), 1023.0f); };
  const uint32_t x = q((s.x - lo.x) * inv_ext.x), y = q((s.y - lo.y) * inv_ext.y), z = q((s.z - lo.z) * inv_ext.z);
  code[i] = expand_bits(x) * 4u + expand_bits(y) * 2u + expand_bits(z);
  idx[i] = (uint32_t)i;
}

// common-prefix length of sorted keys i and j (-1 outside); equal codes
// compare their positions, so every key is distinct
__device__ __forceinline__ int delta(const uint32_t* __restrict__ code, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint32_t a = code[i], b = code[j];
  if (a != b) return __clz(a ^ b);
  return 32 + __clz((uint32_t)i ^ (uint32_t)j);
}

// Node ids: internal nodes 0..n-2 (root 0), leaf j (sorted position) = n-1+j.
__global__ void k_karras(const uint32_t* __restrict__ code, int n, int2* __restrict__ child,
                         int* __restrict__ parent, int8_t* __restrict__ axis) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int d = (delta(code, n, i, i + 1) - delta(code, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = delta(code, n, i, i - d);
  int lmax = 2;
  while (delta(code, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(code, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(code, n, i, j);
  int s = 0;
  for (int div = 2;; div <<= 1) {
    const int t = (l + div - 1) / div;
    if (delta(code, n, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const int gamma = i + s * d + min(d, 0);
  const int first = min(i, j), last = max(i, j);
  const int left = (first == gamma) ? (n - 1 + gamma) : gamma;
  const int right = (last == gamma + 1) ? (n - 1 + gamma + 1) : gamma + 1;
  child[i] = make_int2(left, right);
  parent[left] = i;
  parent[right] = i;
  // split axis: the Morton bit the range splits on (x at bits 3k+2, y 3k+1,
  // z 3k); ranges of equal codes split by position: x
  const int bit = 31 - dnode;
  axis[i] = (int8_t)(dnode >= 32 ? 0 : (bit % 3 == 2 ? 0 : (bit % 3 == 1 ? 1 : 2)));
  if (i == 0) parent[0] = -1;
}

// leaf boxes padded like the host builder; climb while this thread is the
// second to arrive at the parent
__global__ void k_boxes(const float4* __restrict__ cr, const uint32_t* __restrict__ idx, int n,
                        const int2* __restrict__ child, const int* __restrict__ parent, float4* __restrict__ blo,
                        float4* __restrict__ bhi, int* __restrict__ size, int* __restrict__ arrivals) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int leaf = n - 1 + j;
  const float4 s = cr[idx[j]];
  const float pad = 0.002f * s.w + 1e-5f + 0x1p-16f * (fmaxf(fabsf(s.x), fmaxf(fabsf(s.y), fabsf(s.z))) + s.w);  // as the host
  blo[leaf] = make_float4(s.x - s.w - pad, s.y - s.w - pad, s.z - s.w - pad, 0.f);
  bhi[leaf] = make_float4(s.x + s.w + pad, s.y + s.w + pad, s.z + s.w + pad, 0.f);
  size[leaf] = 1;
  __threadfence();
  int node = parent[leaf];
  while (node >= 0) {
    if (atomicAdd(&arrivals[node], 1) == 0) return;  // the sibling's thread finishes this node
    __threadfence();
    const int2 c = child[node];
    const float4 al = blo[c.x], ah = bhi[c.x], bl = blo[c.y], bh = bhi[c.y];
    blo[node] = make_float4(fminf(al.x, bl.x), fminf(al.y, bl.y), fminf(al.z, bl.z), 0.f);
    bhi[node] = make_float4(fmaxf(ah.x, bh.x), fmaxf(ah.y, bh.y), fmaxf(ah.z, bh.z), 0.f);
    size[node] = 1 + size[c.x] + size[c.y];
    __threadfence();
    node = parent[node];
  }
}

// one thread per (node, octant): depth-first position by climbing to the root
__global__ void k_flatten(const float4* __restrict__ cr, const uint32_t* __restrict__ idx, int n,
                          const int2* __restrict__ child, const int* __restrict__ parent,
                          const int8_t* __restrict__ axis, const float4* __restrict__ blo,
                          const float4* __restrict__ bhi, const int* __restrict__ size, BvhNode* __restrict__ out) {
  const int nn = 2 * n - 1;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)nn * 8) return;
  const int oct = (int)(g / nn), x = (int)(g % nn);
  int pos = 0;
  for (int c = x, p = parent[x]; p >= 0; c = p, p = parent[p]) {
    const int2 ch = child[p];
    const bool neg = (oct >> axis[p]) & 1;  // moving toward lower coordinates: right (upper) child first
    const int near = neg ? ch.y : ch.x;
    pos += (c == near) ? 1 : 1 + size[near];
  }
  BvhNode nd;
  nd.skip = pos + size[x];
  if (x >= n - 1) {  // leaf: the sphere itself
    const uint32_t sidx = idx[x - (n - 1)];
    const float4 s = cr[sidx];
    nd.lo[0] = s.x, nd.lo[1] = s.y, nd.lo[2] = s.z;
    nd.hi[0] = s.w * s.w;
    nd.hi[1] = __int_as_float((int)sidx);
    nd.hi[2] = 0.f;
    nd.leaf = kBvhLeafSphere;
  } else {
    const float4 l = blo[x], h = bhi[x];
    nd.lo[0] = l.x, nd.lo[1] = l.y, nd.lo[2] = l.z;
    nd.hi[0] = h.x, nd.hi[1] = h.y, nd.hi[2] = h.z;
    nd.leaf = 0;
  }
  out[(int64_t)oct * nn + pos] = nd;
}

__global__ void k_geom(const float4* __restrict__ cr, const uint32_t* __restrict__ idx, int n,
                       DevSphereG* __restrict__ geom) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const float4 s = cr[idx[j]];
  DevSphereG g;
  g.c[0] = s.x, g.c[1] = s.y, g.c[2] = s.z;
  g.rr = s.w * s.w;
  g.orig = (int32_t)idx[j];
  g.pad[0] = g.pad[1] = g.pad[2] = 0;
  geom[j] = g;
}

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
}

}  // namespace
}  // namespace rtp

// Builds the 8 octant copies (8 * (2n-1) nodes into d_nodes) and the leaf-
// order sphere records (n into d_geom) from d_cr (float4 centre + radius per
// sphere, scene order).  lo / ext: bounding box of the centres.  n >= 2.
extern "C" hipError_t rtp_build_bvh_gpu(const float4* d_cr, int n, float3 lo, float3 ext, rtp::BvhNode* d_nodes,
                                        rtp::DevSphereG* d_geom, hipStream_t stream) {
  using namespace rtp;
  if (n < 2) return hipErrorInvalidValue;
  const int nn = 2 * n - 1;
  uint32_t *code = nullptr, *code2 = nullptr, *idx = nullptr, *idx2 = nullptr;
  int2* child = nullptr;
  int *parent = nullptr, *size = nullptr, *arrivals = nullptr;
  int8_t* axis = nullptr;
  float4 *blo = nullptr, *bhi = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  hipError_t e = hipSuccess;
  auto cleanup = [&]() {
    for (void* p : {(void*)code, (void*)code2, (void*)idx, (void*)idx2, (void*)child, (void*)parent, (void*)size,
                    (void*)arrivals, (void*)axis, (void*)blo, (void*)bhi, temp})
      if (p) (void)hipFree(p);
  };
#define RTP_TRY(x)            \
  do {                        \
    e = (x);                  \
    if (e != hipSuccess) {    \
      cleanup();              \
      return e;               \
    }                         \
  } while (0)
  RTP_TRY(dalloc(&code, n));
  RTP_TRY(dalloc(&code2, n));
  RTP_TRY(dalloc(&idx, n));
  RTP_TRY(dalloc(&idx2, n));
  RTP_TRY(dalloc(&child, n));
  RTP_TRY(dalloc(&parent, nn));
  RTP_TRY(dalloc(&size, nn));
  RTP_TRY(dalloc(&arrivals, n));
  RTP_TRY(dalloc(&axis, n));
  RTP_TRY(dalloc(&blo, nn));
  RTP_TRY(dalloc(&bhi, nn));
  const float3 inv = make_float3(ext.x > 0 ? 1.f / ext.x : 0.f, ext.y > 0 ? 1.f / ext.y : 0.f,
                                 ext.z > 0 ? 1.f / ext.z : 0.f);
  const int tb = 256;
  hipLaunchKernelGGL(k_morton, dim3((n + tb - 1) / tb), dim3(tb), 0, stream, d_cr, n, lo, inv, code, idx);
  RTP_TRY(hipGetLastError());
  RTP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, code, code2, idx, idx2, n, 0, 30, stream));
  RTP_TRY(hipMalloc(&temp, temp_bytes));
  RTP_TRY(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, code, code2, idx, idx2, n, 0, 30, stream));
  hipLaunchKernelGGL(k_karras, dim3((n - 1 + tb - 1) / tb), dim3(tb), 0, stream, code2, n, child, parent, axis);
  RTP_TRY(hipGetLastError());
  RTP_TRY(hipMemsetAsync(arrivals, 0, sizeof(int) * n, stream));
  hipLaunchKernelGGL(k_boxes, dim3((n + tb - 1) / tb), dim3(tb), 0, stream, d_cr, idx2, n, child, parent, blo, bhi,
                     size, arrivals);
  RTP_TRY(hipGetLastError());
  const int64_t work = (int64_t)nn * 8;
  hipLaunchKernelGGL(k_flatten, dim3((unsigned)((work + tb - 1) / tb)), dim3(tb), 0, stream, d_cr, idx2, n, child,
                     parent, axis, blo, bhi, size, d_nodes);
  RTP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_geom, dim3((n + tb - 1) / tb), dim3(tb), 0, stream, d_cr, idx2, n, d_geom);
  RTP_TRY(hipGetLastError());
  RTP_TRY(hipStreamSynchronize(stream));
#undef RTP_TRY
  cleanup();
  return hipSuccess;
}

namespace rtp {
namespace {
// f32 -> f16 bits rounded outward: the nearest half, then stepped toward
// -inf (down) or +inf (up) until its value (decoded by the same instruction
// the walk uses) is on the right side of x; if that fails, an infinity.
__device__ uint32_t half_outward(float x, bool up) {
  uint32_t b = __builtin_bit_cast(uint16_t, (_Float16)x);
  for (int i = 0; i < 4; i++) {
    const float v = (float)__builtin_bit_cast(_Float16, (uint16_t)b);
    if (up ? v >= x : v <= x) return b;
    const bool neg = (b & 0x8000u) != 0, zero = (b & 0x7fffu) == 0;
    if (zero) b = up ? 0x0001u : 0x8001u;
    else if (up) b = neg ? b - 1 : b + 1;
    else b = neg ? b + 1 : b - 1;
  }
  return up ? 0x7c00u : 0xfc00u;
}
__global__ void k_compact(const BvhNode* __restrict__ nodes, int64_t total, uint32_t* __restrict__ cn,
                          int32_t* __restrict__ cidx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const BvhNode nd = nodes[i];
  uint32_t w[4];
  int32_t idx = -1;
  if (nd.leaf == kBvhLeafSphere) {
    w[0] = __float_as_uint(nd.lo[0]);
    w[1] = __float_as_uint(nd.lo[1]);
    w[2] = __float_as_uint(nd.lo[2]);
    w[3] = __float_as_uint(nd.hi[0]) | kCBvhSphereBit;
    idx = __float_as_int(nd.hi[1]);
  } else {
    w[0] = half_outward(nd.lo[0], false) | half_outward(nd.lo[1], false) << 16;
    w[1] = half_outward(nd.lo[2], false) | half_outward(nd.hi[0], true) << 16;
    w[2] = half_outward(nd.hi[1], true) | half_outward(nd.hi[2], true) << 16;
    w[3] = nd.leaf == 0 ? (uint32_t)nd.skip : kCBvhLeafBit | (uint32_t)nd.leaf;
  }
  reinterpret_cast<uint4*>(cn)[i] = make_uint4(w[0], w[1], w[2], w[3]);
  cidx[i] = idx;
}
}  // namespace
}  // namespace rtp

// The walks' compact copy (rtp_layout.hpp kCBvhSphereBit) of `total` BvhNode
// entries (all 8 octant copies): cn gets 4 words per node, cidx one index.
extern "C" hipError_t rtp_compact_bvh(const rtp::BvhNode* d_nodes, int64_t total, uint32_t* d_cn, int32_t* d_cidx,
                                      hipStream_t stream) {
  if (total <= 0) return hipSuccess;
  const int tb = 256;
  hipLaunchKernelGGL(rtp::k_compact, dim3((unsigned)((total + tb - 1) / tb)), dim3(tb), 0, stream, d_nodes, total,
                     d_cn, d_cidx);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  return e;
}
