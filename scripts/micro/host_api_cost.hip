// Host cost of the HIP calls a run makes (launch of a tiny kernel, event record, memset,
// stream wait on an event) while the device is busy: what bounds a run's enqueue rate.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_spin(unsigned long long cycles) {
    const unsigned long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}
__global__ void k_tiny(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }

int main() {
    hipStream_t s, s2;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    int* d;
    hipMalloc(&d, 1 << 20);
    hipEvent_t ev[64];
    for (auto& e : ev) hipEventCreate(&e);
    const int n = 200;
    auto bench = [&](const char* what, auto&& f) {
        k_spin<<<1, 64, 0, s>>>(2000000000ull);   // keep the device busy (~1 s)
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; ++i) f(i);
        auto t1 = std::chrono::steady_clock::now();
        hipStreamSynchronize(s);
        hipStreamSynchronize(s2);
        printf("%-34s %7.2f us per call\n", what, std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
    };
    bench("kernel launch (tiny, 1 block)", [&](int) { k_tiny<<<1, 64, 0, s>>>(d); });
    bench("kernel launch (tiny, 1024 blocks)", [&](int) { k_tiny<<<1024, 256, 0, s>>>(d); });
    bench("hipEventRecord (timing)", [&](int i) { hipEventRecord(ev[i % 64], s); });
    bench("hipMemsetAsync 4 KB", [&](int) { hipMemsetAsync(d, 0, 4096, s); });
    bench("hipStreamWaitEvent (other stream)", [&](int i) { hipEventRecord(ev[i % 64], s); hipStreamWaitEvent(s2, ev[i % 64], 0); });
    bench("launch + event record", [&](int i) { k_tiny<<<1, 64, 0, s>>>(d); hipEventRecord(ev[i % 64], s); });
    return 0;
}
