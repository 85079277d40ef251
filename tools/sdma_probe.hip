// Probe: device -> host copies through hipMemcpyAsync (ROCclr picks a blit kernel or a copy
// engine) against hsa_amd_memory_async_copy (an SDMA engine), alone and beside a compute kernel
// that occupies every CU.  Answers two questions for rt_render's host copies:
// the bandwidth of each path, and how much each slows a kernel running meanwhile.
//
//   hipcc --offload-arch=gfx950 -O2 tools/sdma_probe.hip -o tools/sdma_probe -lhsa-runtime64
//   tools/sdma_probe [MB]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char* m_ = nullptr; hsa_status_string(s_, &m_); std::printf("%s: %s\n", #x, m_ ? m_ : "?"); std::exit(1); } } while (0)

// ~iters dependent f64 FMAs per lane: a fixed amount of VALU work on every CU
__global__ void busy(double* out, int iters) {
    double a = threadIdx.x * 1e-3, b = 1.0000001;
    for (int i = 0; i < iters; ++i) a = a * b + 1e-9;
    if (a == 12345.0) out[blockIdx.x] = a;
}

static hsa_agent_t g_gpu{}, g_cpu{};
static int g_ngpu = 0;
static hsa_status_t find_agents(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && g_ngpu++ == 0) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 192;
    const size_t bytes = mb << 20, piece = 8u << 20;
    CK(hipSetDevice(0));
    void *d = nullptr, *h = nullptr;
    double* dout = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&dout, 1 << 20));
    CK(hipMemset(d, 1, bytes));
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    std::vector<unsigned char> pageable(bytes);
    void* reg = std::aligned_alloc(4096, bytes);
    std::memset(reg, 0, bytes);
    CK(hipHostRegister(reg, bytes, hipHostRegisterDefault));
    hipStream_t sk, sc;
    CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    HK(hsa_iterate_agents(find_agents, nullptr));
    uint32_t emask = 0, pmask = 0;
    HK(hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &emask));
    (void)hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &pmask);
    std::printf("hsa: %d gpu agents; D2H sdma engines available mask 0x%x, preferred 0x%x\n", g_ngpu, emask, pmask);
    hsa_signal_t sig;
    HK(hsa_signal_create(1, 0, nullptr, &sig));

    auto hip_copy = [&](void* dst) {
        for (size_t o = 0; o < bytes; o += piece)
            CK(hipMemcpyAsync(static_cast<char*>(dst) + o, static_cast<char*>(d) + o, std::min(piece, bytes - o),
                              hipMemcpyDeviceToHost, sc));
        CK(hipStreamSynchronize(sc));
    };
    // one engine, pieces chained through one signal (each piece waits for the previous completion)
    auto hsa_copy = [&](void* dst, int engine_bit) {
        const size_t n = (bytes + piece - 1) / piece;
        hsa_signal_store_relaxed(sig, static_cast<hsa_signal_value_t>(n));
        for (size_t o = 0; o < bytes; o += piece) {
            hsa_status_t s = engine_bit
                ? hsa_amd_memory_async_copy_on_engine(static_cast<char*>(dst) + o, g_cpu, static_cast<char*>(d) + o, g_gpu,
                                                      std::min(piece, bytes - o), 0, nullptr, sig,
                                                      static_cast<hsa_amd_sdma_engine_id_t>(engine_bit), true)
                : hsa_amd_memory_async_copy(static_cast<char*>(dst) + o, g_cpu, static_cast<char*>(d) + o, g_gpu,
                                            std::min(piece, bytes - o), 0, nullptr, sig);
            HK(s);
        }
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    };

    const int iters = 200000;
    const int blocks = 256 * 8;
    auto kernel_ms = [&]() {
        hipEvent_t a, b;
        CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        CK(hipEventRecord(a, sk));
        hipLaunchKernelGGL(busy, dim3(blocks), dim3(256), 0, sk, dout, iters);
        CK(hipEventRecord(b, sk));
        return std::make_pair(a, b);
    };
    auto elapsed = [&](std::pair<hipEvent_t, hipEvent_t> e) {
        CK(hipEventSynchronize(e.second));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e.first, e.second));
        return ms;
    };
    // warm up everything
    hip_copy(h);
    hsa_copy(h, 0);
    (void)elapsed(kernel_ms());

    for (int rep = 0; rep < 2; ++rep) {
        std::printf("--- rep %d, %zu MB in 8 MiB pieces\n", rep, mb);
        auto t0 = Clock::now();
        hip_copy(h);
        double t = ms_since(t0);
        std::printf("hipMemcpyAsync -> hipHostMalloc:   %.3f ms  %.1f GB/s\n", t, bytes / t / 1e6);
        t0 = Clock::now();
        hip_copy(reg);
        t = ms_since(t0);
        std::printf("hipMemcpyAsync -> hipHostRegister: %.3f ms  %.1f GB/s\n", t, bytes / t / 1e6);
        t0 = Clock::now();
        hsa_copy(h, 0);
        t = ms_since(t0);
        std::printf("hsa async copy -> hipHostMalloc:   %.3f ms  %.1f GB/s\n", t, bytes / t / 1e6);
        for (int b = 0; b < 16; ++b) {                 // every available engine (its first use sets up its queue)
            if (!(emask & (1u << b))) continue;
            for (int k = 0; k < 2; ++k) {
                t0 = Clock::now();
                hsa_copy(h, 1 << b);
                t = ms_since(t0);
                if (k == 1) std::printf("hsa copy on engine 0x%x -> pinned:  %.3f ms  %.1f GB/s\n", 1 << b, t, bytes / t / 1e6);
            }
        }
        t0 = Clock::now();
        hsa_copy(reg, 0);
        t = ms_since(t0);
        std::printf("hsa async copy -> hipHostRegister: %.3f ms  %.1f GB/s (host pointer)\n", t, bytes / t / 1e6);
        // a compute kernel alone, then beside each copy
        const float alone = elapsed(kernel_ms());
        auto e1 = kernel_ms();
        t0 = Clock::now();
        hip_copy(h);
        const double c1 = ms_since(t0);
        const float with_hip = elapsed(e1);
        auto e2 = kernel_ms();
        t0 = Clock::now();
        hsa_copy(h, 0);
        const double c2 = ms_since(t0);
        const float with_hsa = elapsed(e2);
        std::printf("busy kernel alone %.3f ms; beside hipMemcpyAsync %.3f ms (copy %.3f ms); beside hsa copy %.3f ms "
                    "(copy %.3f ms)\n", alone, with_hip, c1, with_hsa, c2);
    }
    // a rank's row bands into a shared frame: nb pieces of `pb` bytes, `stride` pieces apart on the host
    // (8 ranks: every 8th band), through hipMemcpyAsync per piece, one hipMemcpy2DAsync, and engines
    // driven directly (one, or four round-robin)
    for (size_t pb : {size_t(196608), size_t(786432), size_t(1572864)}) {
        const size_t nb = std::min<size_t>(64, bytes / pb / 8), stride = 8 * pb;
        if (nb < 2) continue;
        auto t0 = Clock::now();
        for (size_t b = 0; b < nb; ++b)
            CK(hipMemcpyAsync(static_cast<char*>(h) + b * stride, static_cast<char*>(d) + b * pb, pb, hipMemcpyDeviceToHost, sc));
        CK(hipStreamSynchronize(sc));
        const double t1 = ms_since(t0);
        t0 = Clock::now();
        CK(hipMemcpy2DAsync(h, stride, d, pb, pb, nb, hipMemcpyDeviceToHost, sc));
        CK(hipStreamSynchronize(sc));
        const double t2 = ms_since(t0);
        double te[2] = {0, 0};
        for (int ne : {1, 4}) {
            t0 = Clock::now();
            hsa_signal_store_relaxed(sig, static_cast<hsa_signal_value_t>(nb));
            for (size_t b = 0; b < nb; ++b)
                HK(hsa_amd_memory_async_copy_on_engine(static_cast<char*>(h) + b * stride, g_cpu, static_cast<char*>(d) + b * pb,
                                                       g_gpu, pb, 0, nullptr, sig,
                                                       static_cast<hsa_amd_sdma_engine_id_t>(1u << (b % ne)), true));
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
            te[ne == 4] = ms_since(t0);
        }
        const double mbt = nb * pb / 1e6;
        std::printf("bands %zu x %zu KB: per-piece hipMemcpyAsync %.3f ms (%.1f GB/s), one 2D copy %.3f ms (%.1f GB/s), "
                    "engine 0 %.3f ms (%.1f GB/s), engines 0-3 %.3f ms (%.1f GB/s)\n", nb, pb >> 10, t1, mbt / t1, t2,
                    mbt / t2, te[0], mbt / te[0], te[1], mbt / te[1]);
    }
    // correctness of the hsa copy into registered memory
    CK(hipMemset(d, 7, bytes));
    CK(hipDeviceSynchronize());
    hsa_copy(reg, 0);
    bool ok = true;
    for (size_t i = 0; i < bytes; i += 4093) ok &= static_cast<unsigned char*>(reg)[i] == 7;
    std::printf("hsa copy into registered memory correct: %s\n", ok ? "yes" : "NO");
    (void)pageable;
    hsa_signal_destroy(sig);
    CK(hipHostUnregister(reg));
    std::free(reg);
    CK(hipHostFree(h));
    CK(hipFree(d));
    CK(hipFree(dout));
    std::printf("done\n");
    return 0;
}
