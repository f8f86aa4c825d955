// Experiment probe: can the host CPU write device memory directly (large-BAR
// mapping of fine-grained device memory), and how fast does a polling kernel
// see it?  Prints one line per check.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void poll_kernel(volatile unsigned* flag, unsigned* out, unsigned expect) {
    unsigned spins = 0;
    while (__hip_atomic_load((unsigned*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != expect && spins < (1u << 26)) ++spins;
    out[0] = spins;
    __hip_atomic_store((unsigned*)out + 1, expect, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
    unsigned* dflag = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&dflag, 4096, hipDeviceMallocFinegrained);
    printf("hipExtMallocWithFlags(fine-grained): %s\n", hipGetErrorString(e));
    if (e != hipSuccess) return 1;
    hipPointerAttribute_t attr;
    e = hipPointerGetAttributes(&attr, dflag);
    printf("attributes: %s type %d hostPointer %p devicePointer %p\n", hipGetErrorString(e), (int)attr.type, attr.hostPointer, attr.devicePointer);
    unsigned* hout = nullptr;
    hipHostMalloc((void**)&hout, 4096, hipHostMallocCoherent | hipHostMallocMapped);
    hout[0] = hout[1] = 0;
    hipMemset(dflag, 0, 4096);
    hipDeviceSynchronize();
    // a CPU store to the device pointer (segfaults here when the BAR is not mapped)
    volatile unsigned* hp = (volatile unsigned*)dflag;
    unsigned* dout = nullptr;
    hipHostGetDevicePointer((void**)&dout, hout, 0);
    for (unsigned it = 1; it <= 5; ++it) {
        hipLaunchKernelGGL(poll_kernel, dim3(1), dim3(64), 0, 0, (volatile unsigned*)dflag, dout, it);
        for (volatile int w = 0; w < 2000000; ++w) {}
        auto t0 = std::chrono::steady_clock::now();
        hp[0] = it;
        __builtin_ia32_sfence();  // (write-combined BAR mapping: push the store out)
        while (__atomic_load_n(&hout[1], __ATOMIC_ACQUIRE) != it) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) { printf("timeout\n"); return 2; }
        }
        auto t1 = std::chrono::steady_clock::now();
        printf("round trip %u: %.2f us (kernel spins %u)\n", it, std::chrono::duration<double, std::micro>(t1 - t0).count(), hout[0]);
        hipDeviceSynchronize();
    }
    // the same with the doorbell in pinned host memory (the kernel polls across PCIe)
    unsigned* hflag = nullptr;
    hipHostMalloc((void**)&hflag, 4096, hipHostMallocCoherent | hipHostMallocMapped);
    hflag[0] = 0;
    unsigned* dhflag = nullptr;
    hipHostGetDevicePointer((void**)&dhflag, hflag, 0);
    for (unsigned it = 11; it <= 15; ++it) {
        hipLaunchKernelGGL(poll_kernel, dim3(1), dim3(64), 0, 0, (volatile unsigned*)dhflag, dout, it);
        for (volatile int w = 0; w < 2000000; ++w) {}
        auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(&hflag[0], it, __ATOMIC_RELEASE);
        while (__atomic_load_n(&hout[1], __ATOMIC_ACQUIRE) != it) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) { printf("timeout\n"); return 2; }
        }
        auto t1 = std::chrono::steady_clock::now();
        printf("host-memory doorbell round trip %u: %.2f us (kernel spins %u)\n", it, std::chrono::duration<double, std::micro>(t1 - t0).count(), hout[0]);
        hipDeviceSynchronize();
    }
    return 0;
}
