// FETCH_SIZE / WRITE_SIZE calibration for the denoiser's access widths (MI355X_MICROARCH.md, HBM:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Streams a 512 MiB buffer (past the 256 MiB Infinity Cache) once per kernel with
// 4-, 8- and 16-byte loads per lane, and writes it back with the same widths; rocprofv3 --pmc
// FETCH_SIZE / WRITE_SIZE (separate runs) per dispatch / the known byte count = the factor.
#include <hip/hip_runtime.h>
#include <cstdio>

template <class T>
__global__ __launch_bounds__(256) void k_read(const T *__restrict__ in, size_t n, float *sink) {
    float acc = 0.0f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const T v = in[i];
        acc += reinterpret_cast<const float *>(&v)[0];
    }
    if (acc == 12345.678f) sink[0] = acc;  // keeps the loads
}
template <class T>
__global__ __launch_bounds__(256) void k_write(T *__restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) out[i] = T{};
}

int main() {
    const size_t bytes = 512ull << 20;
    char *buf;
    float *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    const dim3 g(4096), b(256);
    hipLaunchKernelGGL(k_read<float>, g, b, 0, 0, (const float *)buf, bytes / 4, sink);
    hipLaunchKernelGGL(k_read<float2>, g, b, 0, 0, (const float2 *)buf, bytes / 8, sink);
    hipLaunchKernelGGL(k_read<float4>, g, b, 0, 0, (const float4 *)buf, bytes / 16, sink);
    hipLaunchKernelGGL(k_write<float>, g, b, 0, 0, (float *)buf, bytes / 4);
    hipLaunchKernelGGL(k_write<float4>, g, b, 0, 0, (float4 *)buf, bytes / 16);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("calibration: %zu bytes per kernel\n", bytes);
    hipFree(buf);
    hipFree(sink);
    return 0;
}
