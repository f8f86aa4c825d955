// Probe: does v_pk_maximum3_f16 order non-negative int16 bit patterns like
// integers (normal and denormal f16 ranges)?  Prints mismatch counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
__global__ void k(const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t r;
    asm volatile("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
    o[i] = r;
}
static uint32_t mx(uint32_t x, uint32_t y, uint32_t z, int sh) {
    uint32_t a = (x >> sh) & 0xFFFF, b = (y >> sh) & 0xFFFF, c = (z >> sh) & 0xFFFF;
    uint32_t m = a > b ? a : b;
    return m > c ? m : c;
}
int main() {
    const int n = 1 << 22;
    for (int range = 0; range < 2; ++range) {
        uint32_t lo = range ? 0x0000 : 0x0400, hi = range ? 0x0800 : 0x7BFF;
        std::vector<uint32_t> a(n), b(n), c(n), o(n);
        srand(7 + range);
        auto rnd = [&]() { return lo + (uint32_t)(rand() % (hi - lo + 1)); };
        for (int i = 0; i < n; ++i) {
            a[i] = rnd() | (rnd() << 16);
            b[i] = (i & 7) == 0 ? a[i] : (rnd() | (rnd() << 16));
            c[i] = rnd() | (rnd() << 16);
        }
        uint32_t *da, *db, *dc, *dout;
        hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&dout, n * 4);
        hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
        hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
        hipMemcpy(dc, c.data(), n * 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, da, db, dc, dout, n);
        hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost);
        long bad = 0;
        for (int i = 0; i < n; ++i) {
            uint32_t want = mx(a[i], b[i], c[i], 0) | (mx(a[i], b[i], c[i], 16) << 16);
            if (o[i] != want) { if (bad < 3) printf("  range %d: %08x %08x %08x -> %08x want %08x\n", range, a[i], b[i], c[i], o[i], want); ++bad; }
        }
        printf("range [%04x,%04x]: %ld of %d differ\n", lo, hi, bad, n);
        hipFree(da); hipFree(db); hipFree(dc); hipFree(dout);
    }
    return 0;
}
