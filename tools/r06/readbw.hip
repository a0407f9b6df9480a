// Read-bandwidth probe for the weight-gradient pass's access pattern (tools only, not part of the library):
// 2.4 GB streamed by 766 workgroups of 256 threads, (a) 4-B loads, each wave instruction one 256-B row segment,
// 32 loads in flight per thread (the pattern of wgrad_bf3_kernel's staging), (b) the same bytes as 16-B loads.
// hipcc --offload-arch=gfx950 -O3 tools/r06/readbw.hip -o tools/r06/readbw && ./tools/r06/readbw
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void read_dword(const float* __restrict__ p, size_t n, float* out) {
  const size_t chunk = (n / gridDim.x) & ~(size_t)8191;
  const float* b = p + blockIdx.x * chunk;
  float acc = 0.f;
  for (size_t r = 0; r + 8192 <= chunk; r += 8192) {  // 8192 floats = 32 rows of 256 threads (32 KB in flight)
    float v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = b[r + k * 256 + threadIdx.x];
#pragma unroll
    for (int k = 0; k < 32; ++k) acc += v[k];
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void read_dwordx4(const float4* __restrict__ p, size_t n4, float* out) {
  const size_t chunk = (n4 / gridDim.x) & ~(size_t)2047;
  const float4* b = p + blockIdx.x * chunk;
  float acc = 0.f;
  for (size_t r = 0; r + 2048 <= chunk; r += 2048) {  // 32 KB in flight
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = b[r + k * 256 + threadIdx.x];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

int main() {
  const size_t bytes = (size_t)2400 << 20;
  const size_t n = bytes / 4;
  float *p, *out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 4096) != hipSuccess) return 1;
  (void)hipMemset(p, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int grid : {766, 1532, 3064}) {
    for (int kind = 0; kind < 2; ++kind) {
      float best = 1e30f;
      for (int rep = 0; rep < 6; ++rep) {
        (void)hipEventRecord(e0);
        if (kind == 0) read_dword<<<grid, 256>>>(p, n, out);
        else read_dwordx4<<<grid, 256>>>((const float4*)p, n / 4, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
      }
      // bytes actually read: whole 8192-float (32-KB) steps of each workgroup's chunk
      const size_t per = kind == 0 ? ((n / grid) & ~(size_t)8191) * 4 : ((n / 4 / grid) & ~(size_t)2047) * 16;
      printf("grid %5d %-8s %.3f ms  %.2f TB/s\n", grid, kind == 0 ? "dword" : "dwordx4", best,
             (double)per * grid / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
