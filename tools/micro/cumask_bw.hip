// tools/micro/cumask_bw.hip -- where the workgroups of a CU-masked stream land (XCC id and
// HW_ID of each workgroup), and the float4 copy bandwidth a masked subset of CUs reaches.
// Build: hipcc --offload-arch=gfx950 -O2 -o build/cumask_bw tools/micro/cumask_bw.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

__global__ __launch_bounds__(1024) void where_kernel(unsigned long long spin, uint32_t *out) {
  extern __shared__ unsigned lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned acc = threadIdx.x;
  while (__builtin_amdgcn_s_memtime() - t0 < spin) {
    lds[threadIdx.x] = acc;
    acc += lds[(threadIdx.x + 1) & 1023];
  }
  if (threadIdx.x == 0) {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw + (acc == 0xdeadbeef ? 1u : 0u);
  }
}

// persistent grid-stride float4 copy
__global__ __launch_bounds__(1024) void copy_kernel(const float4 *__restrict__ a, float4 *__restrict__ b,
                                                    size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static std::vector<uint32_t> mask_range(int lo, int hi, int total) {
  std::vector<uint32_t> m((total + 31) / 32, 0u);
  for (int i = lo; i < hi; i++) m[i / 32] |= 1u << (i % 32);
  return m;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  uint32_t *out;
  CK(hipMalloc(&out, 8 * 4096));
  CK(hipFuncSetAttribute((const void *)where_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
  std::vector<uint32_t> h(2 * 4096);
  for (int n : {32, 64, 128}) {
    auto m = mask_range(0, n, ncu);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    where_kernel<<<n, 1024, 150 * 1024, s>>>(200000, out);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), out, 8 * n, hipMemcpyDeviceToHost));
    int cnt[16] = {0};
    std::set<uint32_t> ids;
    for (int i = 0; i < n; i++) {
      cnt[h[2 * i] & 15]++;
      ids.insert((h[2 * i] << 16) | ((h[2 * i + 1] >> 8) & 0xFFFF));
    }
    printf("first %3d bits: workgroups per XCC:", n);
    for (int x = 0; x < 8; x++) printf(" %d", cnt[x]);
    printf("  (distinct XCC+CU/SE ids %zu)\n", ids.size());
    CK(hipStreamDestroy(s));
  }
  // copy bandwidth: 2 GiB each way
  const size_t n4 = (size_t)1 << 27;   // float4 elements = 2 GiB
  float4 *a, *b;
  CK(hipMalloc(&a, n4 * 16));
  CK(hipMalloc(&b, n4 * 16));
  CK(hipMemset(a, 0, n4 * 16));
  for (int n : {64, 128, 160, 192, 224, 256}) {
    auto m = mask_range(0, n, ncu);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    copy_kernel<<<n, 1024, 0, s>>>(a, b, n4);
    CK(hipStreamSynchronize(s));
    double best = 1e9;
    for (int r = 0; r < 3; r++) {
      auto t0 = std::chrono::steady_clock::now();
      copy_kernel<<<n * 2, 1024, 0, s>>>(a, b, n4);
      CK(hipStreamSynchronize(s));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("copy on first %3d CUs: %.2f TB/s (read + write)\n", n, 2.0 * n4 * 16 / (best * 1e-3) / 1e12);
    CK(hipStreamDestroy(s));
  }
  printf("done\n");
  return 0;
}
