// pow5_check.cpp -- pins rtp_device.hpp pow5_exact, the x^5 of schlick
// (EmitWorklet.h:153-158, the reference's pow((double)(1 - cosine), 5.0)),
// for every float x with bit pattern in [lo, hi] (multi-threaded).  The
// formula is restated here with the host's fma (IEEE, exact like the
// device's v_fma_f64).
//   pow5_check cr <lo_hex> <hi_hex>: pow5_exact(x) == the correctly rounded
//       x^5 (x^5 in binary128, 113 bits, rounded to double)
//   pow5_check schlick <ior> <lo_hex> <hi_hex>: the float schlick value
//       (float)(r0 + (1 - r0) * p) with p = glibc pow(x, 5.0) (the reference)
//       equals the one with p = pow5_exact(x), r0 = ((1 - ior)/(1 + ior))^2
//   prints "mismatches N first 0x... of M"
#include <quadmath.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double pow5_exact(double x) {  // = rtp_device.hpp pow5_exact
  const double x2 = x * x;
  const double h = x2 * x2;
  const double l = std::fma(x2, x2, -h);
  const double p = h * x;
  const double e = std::fma(h, x, -p);
  return p + (e + l * x);
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const std::string mode = argv[1];
  const bool sch = mode == "schlick";
  if (sch && argc < 5) return 2;
  const float ior = sch ? (float)atof(argv[2]) : 0.f;
  float r0 = (1 - ior) / (1 + ior);
  r0 = r0 * r0;
  const int a0 = sch ? 3 : 2;
  const uint32_t lo = (uint32_t)strtoul(argv[a0], nullptr, 16), hi = (uint32_t)strtoul(argv[a0 + 1], nullptr, 16);
  const unsigned nt = std::max(1u, std::thread::hardware_concurrency());
  std::atomic<uint64_t> bad{0}, n{0};
  std::atomic<uint32_t> first{0xffffffffu};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++)
    th.emplace_back([&, t] {
      uint64_t b = 0, c = 0;
      for (uint64_t u = (uint64_t)lo + t; u <= hi; u += nt) {
        float xf;
        const uint32_t bits = (uint32_t)u;
        std::memcpy(&xf, &bits, 4);
        const double x = (double)xf;
        bool same;
        if (sch) {
          const float want = (float)(r0 + (1 - r0) * std::pow(x, 5.0));
          const float got = (float)(r0 + (1 - r0) * pow5_exact(x));
          same = std::memcmp(&want, &got, 4) == 0 || (want != want && got != got);
        } else {
          const __float128 X = x;
          const double want = (double)(X * X * X * X * X), got = pow5_exact(x);
          same = std::memcmp(&want, &got, 8) == 0 || (want != want && got != got);
        }
        c++;
        if (!same) {
          b++;
          uint32_t f = first.load();
          while (bits < f && !first.compare_exchange_weak(f, bits)) {
          }
        }
      }
      bad += b;
      n += c;
    });
  for (auto& x : th) x.join();
  printf("mismatches %llu first 0x%08x of %llu\n", (unsigned long long)bad.load(), first.load(),
         (unsigned long long)n.load());
  return 0;
}
