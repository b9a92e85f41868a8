// FETCH_SIZE calibration for chain_estep_ck_kernel's observation reads
// (profiles/pmc_traffic.json, VERDICT r05 item 1's traffic check): the
// kernel's access pattern alone -- 16 sequences per wave, the four lanes of a
// sequence loading the same int4 (four steps) per chunk, chunks in order --
// over config 4's [131072][1024] int32 array (512 MiB), forward then backward.
// Bytes actually needed: 2 x 512 MiB.  Run under rocprofv3 --pmc FETCH_SIZE.
// Paced like the kernel: two waves per SIMD (70 KB of LDS per 4-wave block)
// and ~5.8K cycles between a wave's chunks (s_sleep), so that lines stay in L2
// about as long as they do there.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void obs_read(const int* __restrict__ obs, int T, unsigned* out) {
  extern __shared__ unsigned pad[];
  if (threadIdx.x == 999) pad[0] = 0;           // the LDS only limits residency
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long grp = (long)blockIdx.x * 4 + wave;
  const int j = lane & 15;
  const int* orow = obs + (grp * 16 + j) * (long)T;
  unsigned acc = 0;
  for (int c = 0; c < T / 4; c++) {               // forward
    const int4 v = *reinterpret_cast<const int4*>(orow + 4 * c);
    acc = acc * 31u + (unsigned)(v.x ^ v.y ^ v.z ^ v.w);
    __builtin_amdgcn_s_sleep(90);
  }
  for (int c = T / 4 - 1; c >= 0; c--) {          // backward
    const int4 v = *reinterpret_cast<const int4*>(orow + 4 * c);
    acc = acc * 37u + (unsigned)(v.x + v.y + v.z + v.w);
    __builtin_amdgcn_s_sleep(90);
  }
  out[grp * 64 + lane] = acc;
}

int main() {
  const long B = 131072;
  const int T = 1024;
  int* obs = nullptr;
  unsigned* out = nullptr;
  if (hipMalloc(&obs, B * T * sizeof(int)) != hipSuccess || hipMalloc(&out, B / 16 * 64 * sizeof(unsigned)) != hipSuccess) return 1;
  hipMemset(obs, 1, B * T * sizeof(int));
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&obs_read), hipFuncAttributeMaxDynamicSharedMemorySize, 70 * 1024) != hipSuccess) return 3;
  for (int it = 0; it < 1; it++) hipLaunchKernelGGL(obs_read, dim3((unsigned)(B / 64)), dim3(256), 70 * 1024, 0, obs, T, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(obs_read, dim3((unsigned)(B / 64)), dim3(256), 70 * 1024, 0, obs, T, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("obs_read: %.3f ms, needed %.1f MiB (2 passes)\n", ms, 2.0 * B * T * 4 / 1048576.0);
  return 0;
}
