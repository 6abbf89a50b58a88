// tools/micro/cumask.hip -- does a CU-masked stream confine a kernel to its CUs on this GPU,
// and do two kernels on disjoint masks run side by side?
//   hog_kernel : 1024 threads + 150 KB LDS (one workgroup per CU, like the persistent decode),
//                each workgroup busy-waits `spin` shader-clock ticks
//   small_kernel: 512 threads + 64 KB LDS workgroups (like the search), same busy wait
// A launch of G hog workgroups on a stream whose mask enables C CUs takes ceil(G / C) spins.
// Build: hipcc --offload-arch=gfx950 -O2 -o build/cumask tools/micro/cumask.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(1024) void hog_kernel(unsigned long long spin, unsigned *out) {
  extern __shared__ unsigned lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned acc = threadIdx.x;
  while (__builtin_amdgcn_s_memtime() - t0 < spin) {
    lds[threadIdx.x] = acc;
    acc += lds[(threadIdx.x + 1) & 1023];
  }
  if (acc == 0xdeadbeef) out[0] = acc;
}

__global__ __launch_bounds__(512) void small_kernel(unsigned long long spin, unsigned *out) {
  extern __shared__ unsigned lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned acc = threadIdx.x;
  while (__builtin_amdgcn_s_memtime() - t0 < spin) {
    lds[threadIdx.x] = acc;
    acc += lds[(threadIdx.x + 1) & 511];
  }
  if (acc == 0xdeadbeef) out[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static std::vector<uint32_t> mask_first(int n, int total) {
  std::vector<uint32_t> m((total + 31) / 32, 0u);
  for (int i = 0; i < n; i++) m[i / 32] |= 1u << (i % 32);
  return m;
}
static std::vector<uint32_t> mask_spread(int n, int total, bool complement) {
  std::vector<uint32_t> m((total + 31) / 32, 0u);
  for (int i = 0; i < total; i++) {
    const bool on = ((long)(i + 1) * n / total) > ((long)i * n / total);
    if (on != complement) m[i / 32] |= 1u << (i % 32);
  }
  return m;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  printf("CUs %d\n", ncu);
  unsigned *out;
  CK(hipMalloc(&out, 64));
  CK(hipFuncSetAttribute((const void *)hog_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
  CK(hipFuncSetAttribute((const void *)small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
  const unsigned long long spin = 2000000;   // shader clock (~2 GHz): ~1 ms
  auto timed = [&](auto fn) {
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    fn();
    CK(hipDeviceSynchronize());
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  hipStream_t s0;
  CK(hipStreamCreate(&s0));
  hog_kernel<<<ncu, 1024, 150 * 1024, s0>>>(1000, out);
  printf("hog grid %d, unmasked: %.2f ms (1 spin = 1 ms)\n", ncu,
         timed([&] { hog_kernel<<<ncu, 1024, 150 * 1024, s0>>>(spin, out); }));
  for (int n : {32, 64, 128, 192}) {
    for (int kind = 0; kind < 2; kind++) {
      auto m = kind ? mask_spread(n, ncu, false) : mask_first(n, ncu);
      hipStream_t s;
      CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
      hog_kernel<<<1, 1024, 150 * 1024, s>>>(1000, out);
      const double t1 = timed([&] { hog_kernel<<<n, 1024, 150 * 1024, s>>>(spin, out); });
      const double t2 = timed([&] { hog_kernel<<<2 * n, 1024, 150 * 1024, s>>>(spin, out); });
      const double t4 = timed([&] { hog_kernel<<<4 * n, 1024, 150 * 1024, s>>>(spin, out); });
      std::vector<uint32_t> got(m.size(), 0u);
      CK(hipExtStreamGetCUMask(s, (uint32_t)got.size(), got.data()));
      int pc = 0;
      for (uint32_t w : got) pc += __builtin_popcount(w);
      printf("mask %-6s %3d CUs (get: %d, word0 %08x): hog grid n %.2f ms, 2n %.2f, 4n %.2f\n",
             kind ? "spread" : "first", n, pc, got[0], t1, t2, t4);
      CK(hipStreamDestroy(s));
    }
  }
  // disjoint masks side by side: hog on D spread CUs, small on the complement
  for (int d : {128, 160}) {
    auto ma = mask_spread(d, ncu, false), mb = mask_spread(d, ncu, true);
    hipStream_t sa, sb;
    CK(hipExtStreamCreateWithCUMask(&sa, (uint32_t)ma.size(), ma.data()));
    CK(hipExtStreamCreateWithCUMask(&sb, (uint32_t)mb.size(), mb.data()));
    const int nb = 2 * (ncu - d);    // two small workgroups per CU of the complement
    small_kernel<<<1, 512, 64 * 1024, sb>>>(1000, out);
    hog_kernel<<<1, 1024, 150 * 1024, sa>>>(1000, out);
    const double ta = timed([&] { hog_kernel<<<d, 1024, 150 * 1024, sa>>>(spin, out); });
    const double tb = timed([&] { small_kernel<<<nb, 512, 64 * 1024, sb>>>(spin, out); });
    const double tab = timed([&] {
      hog_kernel<<<d, 1024, 150 * 1024, sa>>>(spin, out);
      small_kernel<<<nb, 512, 64 * 1024, sb>>>(spin, out);
    });
    const double tba = timed([&] {
      small_kernel<<<4 * nb, 512, 64 * 1024, sb>>>(spin / 4, out);
      hog_kernel<<<d, 1024, 150 * 1024, sa>>>(spin, out);
    });
    printf("D %d: hog alone %.2f, small alone %.2f, both %.2f, small-first both %.2f ms\n", d, ta, tb,
           tab, tba);
    // unmasked streams: small kernel first fills every CU, then the hog
    const double tun = timed([&] {
      small_kernel<<<4 * ncu * 2, 512, 64 * 1024, s0>>>(spin / 4, out);
      hog_kernel<<<d, 1024, 150 * 1024, sa>>>(spin, out);
    });
    printf("D %d: unmasked small (4 waves of 2/CU) + masked hog %.2f ms\n", d, tun);
    CK(hipStreamDestroy(sa));
    CK(hipStreamDestroy(sb));
  }
  printf("done\n");
  return 0;
}
