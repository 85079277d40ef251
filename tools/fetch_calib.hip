// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths the
// wavefront kernels use (MI355X_MICROARCH.md: FETCH_SIZE reads half the bytes of
// a 16-B-per-lane streaming read; other widths are uncalibrated).  Each kernel
// streams a 1 GiB buffer (far beyond L2 and the 256 MiB Infinity Cache) once,
// with 4, 8 or 16 bytes per lane per load, or writes it with that width.
// Run under `rocprofv3 --pmc FETCH_SIZE` (then WRITE_SIZE, a separate pass):
// bytes moved / (counter x 1024) is the factor for that width.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <class T>
__global__ void read_stream(const T* __restrict__ p, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x) {
        const T v = __builtin_nontemporal_load(p + i);
        if constexpr (sizeof(T) == 4) acc ^= v; else acc ^= v.x;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;      // keeps the loads; practically never stores
}

template <class T>
__global__ void write_stream(T* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x) {
        __builtin_nontemporal_store(static_cast<T>(static_cast<unsigned>(i)), p + i);
    }
}

typedef unsigned U2 __attribute__((ext_vector_type(2)));
typedef unsigned U4 __attribute__((ext_vector_type(4)));

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

int main() {
    const size_t bytes = size_t(1) << 30;
    void* buf = nullptr;
    unsigned* out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 1, bytes));
    const dim3 grid(256 * 16), block(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(read_stream<unsigned>, grid, block, 0, 0, static_cast<const unsigned*>(buf), bytes / 4, out);
        hipLaunchKernelGGL(read_stream<U2>, grid, block, 0, 0, static_cast<const U2*>(buf), bytes / 8, out);
        hipLaunchKernelGGL(read_stream<U4>, grid, block, 0, 0, static_cast<const U4*>(buf), bytes / 16, out);
        hipLaunchKernelGGL(write_stream<unsigned>, grid, block, 0, 0, static_cast<unsigned*>(buf), bytes / 4);
        hipLaunchKernelGGL(write_stream<U2>, grid, block, 0, 0, static_cast<U2*>(buf), bytes / 8);
        hipLaunchKernelGGL(write_stream<U4>, grid, block, 0, 0, static_cast<U4*>(buf), bytes / 16);
    }
    CK(hipDeviceSynchronize());
    std::printf("fetch_calib: 6 kernels x 2 reps, %zu bytes each\n", bytes);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
