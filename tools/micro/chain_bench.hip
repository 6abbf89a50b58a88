// Micro-benchmark: cycles for a 2048-term sequential fp32 sum read from LDS (one wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)

template <int V>
__global__ void chain(const float *g, float *out, long long *cyc) {
  __shared__ float t[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) t[i] = g[i];
  __syncthreads();
  const int r = threadIdx.x * 7 % 512;
  const float *q = t + r;
  long long c0 = clock64();
  float acc = 0.0f;
  if (V == 0) {
#pragma unroll 8
    for (int k = 0; k < 2048; k++) acc = acc + q[k];
  } else if (V == 1) {
    float nxt[8];
    for (int k = 0; k < 8; k++) nxt[k] = q[k];
    for (int j = 0; j < 2048; j += 8) {
      float cur[8];
#pragma unroll
      for (int k = 0; k < 8; k++) cur[k] = nxt[k];
      if (j + 8 < 2048) {
#pragma unroll
        for (int k = 0; k < 8; k++) nxt[k] = q[j + 8 + k];
      }
#pragma unroll
      for (int k = 0; k < 8; k++) acc = acc + cur[k];
    }
  } else if (V == 2) {   // register-only chain (latency of dependent adds)
    float x = q[0];
#pragma unroll 16
    for (int k = 0; k < 2048; k++) acc = acc + x;
  } else if (V == 3) {   // float4 reads where aligned (r multiple of 4 here not guaranteed)
    const float *qa = t + (r & ~3);
#pragma unroll 4
    for (int k = 0; k < 2048; k += 4) {
      const float4 v = *reinterpret_cast<const float4 *>(qa + k);
      acc = acc + v.x; acc = acc + v.y; acc = acc + v.z; acc = acc + v.w;
    }
  }
  else if (V == 4) {   // float4 reads, next 16 terms in flight while 16 are added
    const float *qa = t + (r & ~3);
    float4 n0 = *reinterpret_cast<const float4 *>(qa), n1 = *reinterpret_cast<const float4 *>(qa + 4),
           n2 = *reinterpret_cast<const float4 *>(qa + 8), n3 = *reinterpret_cast<const float4 *>(qa + 12);
    for (int k = 0; k < 2048; k += 16) {
      const float4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
      if (k + 16 < 2048) {
        n0 = *reinterpret_cast<const float4 *>(qa + k + 16);
        n1 = *reinterpret_cast<const float4 *>(qa + k + 20);
        n2 = *reinterpret_cast<const float4 *>(qa + k + 24);
        n3 = *reinterpret_cast<const float4 *>(qa + k + 28);
      }
      acc = acc + c0.x; acc = acc + c0.y; acc = acc + c0.z; acc = acc + c0.w;
      acc = acc + c1.x; acc = acc + c1.y; acc = acc + c1.z; acc = acc + c1.w;
      acc = acc + c2.x; acc = acc + c2.y; acc = acc + c2.z; acc = acc + c2.w;
      acc = acc + c3.x; acc = acc + c3.y; acc = acc + c3.z; acc = acc + c3.w;
    }
  } else if (V == 5) {   // two independent chains interleaved (latency sharing)
    float acc2 = 0.0f;
    const float *q2 = q + 1024;
#pragma unroll 8
    for (int k = 0; k < 1024; k++) { acc = acc + q[k]; acc2 = acc2 + q2[k]; }
    acc += acc2;
  }
  long long c1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

int main() {
  float *g, *o; long long *c;
  hipMalloc(&g, 8192 * 4); hipMalloc(&o, 1 << 20); hipMalloc(&c, 8 * 64);
  hipMemset(g, 0, 8192 * 4);
  long long h[64];
  auto run = [&](auto k, const char *name, int threads, int blocks) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, g, o, c);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, g, o, c);
    hipDeviceSynchronize();
    hipMemcpy(h, c, 8 * blocks, hipMemcpyDeviceToHost);
    printf("%-28s threads %4d: %lld cycles (%.2f per term)\n", name, threads, h[0], h[0] / 2048.0);
  };
  run(chain<0>, "lds unroll8", 64, 1);
  run(chain<1>, "lds pipelined8", 64, 1);
  run(chain<2>, "register chain", 64, 1);
  run(chain<3>, "lds float4", 64, 1);
  run(chain<4>, "lds float4 pipelined", 64, 1);
  run(chain<5>, "2 chains x 1024 interleaved", 64, 1);
  run(chain<0>, "lds unroll8 (4 waves)", 256, 1);
  run(chain<3>, "lds float4 (4 waves)", 256, 1);
  return 0;
}
