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

int device_side();

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
    return device_side();
}
// (appended) device-side cost of the packets between kernels: N tiny kernels alone, and with
// an event record (timing / no timing) or a wait on a completed event of another stream after
// each; all enqueued behind a spin kernel, timed by events around them
int device_side() {
    hipStream_t s, s2;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    int* d;
    hipMalloc(&d, 4096);
    hipEvent_t t0, t1, et, en, done;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    hipEventCreate(&et);
    hipEventCreateWithFlags(&en, hipEventDisableTiming);
    hipEventCreateWithFlags(&done, hipEventDisableTiming);
    k_tiny<<<1, 64, 0, s2>>>(d);
    hipEventRecord(done, s2);
    hipStreamSynchronize(s2);
    const int n = 100;
    for (int mode = 0; mode < 4; ++mode) {
        k_spin<<<1, 64, 0, s>>>(200000000ull);
        hipEventRecord(t0, s);
        for (int i = 0; i < n; ++i) {
            k_tiny<<<1, 64, 0, s>>>(d);
            if (mode == 1) hipEventRecord(et, s);
            if (mode == 2) hipEventRecord(en, s);
            if (mode == 3) hipStreamWaitEvent(s, done, 0);
        }
        hipEventRecord(t1, s);
        hipEventSynchronize(t1);
        float ms = 0;
        hipEventElapsedTime(&ms, t0, t1);
        const char* what[] = {"tiny kernels alone", "+ timing event record", "+ no-timing event record",
                              "+ wait on a completed event"};
        printf("device: %-28s %7.2f us per kernel\n", what[mode], ms * 1e3 / n);
    }
    return 0;
}
