// Bandwidth ceiling of ONE launch with the env step's shape (tools only, not part of the library): 8192 waves
// (2048 workgroups of 4), each reading 2,816 B and writing 8,448 B contiguous per wave (the ER-200 env step's PMC
// bytes: 23.4 MB read, 68.5 MB written per launch), against an empty launch of the same grid.  Back-to-back
// launches, each timed with events; the median of 200.
// hipcc --offload-arch=gfx950 -O3 tools/r06/envbw.hip -o tools/r06/envbw && ./tools/r06/envbw
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int WR4 = 8448 / 16;            // float4 writes per wave (528: 8 full wave stores + 16 lanes)

__global__ __launch_bounds__(256) void shape_kernel(const float4* __restrict__ in, float4* __restrict__ out, int waves) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= waves) return;
  const float4* src = in + (size_t)w * 176;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = lane; i < 176; i += 64) {  // 2,816 B
    const float4 v = src[i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  float4* dst = out + (size_t)w * WR4;
  for (int i = lane; i < WR4; i += 64) dst[i] = a;
}

__global__ __launch_bounds__(256) void empty_kernel(float* out, int waves) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= waves && out) out[0] = 1.f;
}

int main() {
  const int waves = 8192, grid = waves / 4;
  float4 *in, *out;
  if (hipMalloc(&in, (size_t)waves * 176 * 16) != hipSuccess || hipMalloc(&out, (size_t)waves * WR4 * 16) != hipSuccess)
    return 1;
  (void)hipMemset(in, 0, (size_t)waves * 176 * 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int kind = 0; kind < 2; ++kind) {
    std::vector<float> t;
    for (int rep = 0; rep < 220; ++rep) {
      (void)hipEventRecord(e0);
      if (kind == 0) shape_kernel<<<grid, 256>>>(in, out, waves);
      else empty_kernel<<<grid, 256>>>(nullptr, waves);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 20) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2] * 1e3, mn = t[0] * 1e3;
    const double bytes = (double)waves * (176 * 16 + WR4 * 16);
    printf("%-6s median %.2f us  min %.2f us  %.2f TB/s at the median (%.1f MB per launch)\n",
           kind == 0 ? "shape" : "empty", med, mn, kind == 0 ? bytes / (med * 1e-6) / 1e12 : 0.0, bytes / 1e6);
  }
  return 0;
}
