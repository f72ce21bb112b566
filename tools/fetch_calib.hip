// Calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the access pattern of
// k_env_step: SoA rows, one 4-byte element per lane per row, fully coalesced
// (256 B per wave per row).  The MI355X guide only calibrates 16-B/lane
// streams (FETCH_SIZE = 1/2 of the bytes there); this kernel has a known byte
// count in OUR width so tools/traffic_report.py can derive the factor.
//   k_calib_read : reads ROWS rows of N floats, writes 1 row   (read bytes known)
//   k_calib_write: reads 1 row, writes ROWS rows               (write bytes known)
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ROWS = 24;
constexpr int BLOCK = 256;

__global__ __launch_bounds__(BLOCK) void k_calib_read(const float* __restrict__ x, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < ROWS; r++) s += x[r * n + i];
  y[i] = s;
}

__global__ __launch_bounds__(BLOCK) void k_calib_write(const float* __restrict__ x, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
#pragma unroll
  for (int r = 0; r < ROWS; r++) y[r * n + i] = v + (float)r;
}

#define CK(e)                                                              \
  do {                                                                     \
    hipError_t err_ = (e);                                                 \
    if (err_ != hipSuccess) {                                              \
      std::fprintf(stderr, "%s: %s\n", #e, hipGetErrorString(err_));       \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const long n = 65536L * 16;  // 4 MiB per row, 96 MiB per 24-row pass: past the per-XCD L2
  float *a, *b;
  CK(hipMalloc(&a, sizeof(float) * ROWS * n));
  CK(hipMalloc(&b, sizeof(float) * ROWS * n));
  CK(hipMemset(a, 0, sizeof(float) * ROWS * n));
  CK(hipMemset(b, 0, sizeof(float) * ROWS * n));
  const dim3 grid((unsigned)((n + BLOCK - 1) / BLOCK));
  for (int it = 0; it < 5; it++) {
    k_calib_read<<<grid, BLOCK>>>(a, b, n);
    k_calib_write<<<grid, BLOCK>>>(b, a, n);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::printf("{\"n\": %ld, \"rows\": %d, \"read_bytes_k_calib_read\": %ld, \"write_bytes_k_calib_read\": %ld, "
              "\"read_bytes_k_calib_write\": %ld, \"write_bytes_k_calib_write\": %ld}\n",
              n, ROWS, 4L * ROWS * n, 4L * n, 4L * n, 4L * ROWS * n);
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
