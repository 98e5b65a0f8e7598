// Lab: host cost of the executor's HIP calls (empty kernel launch with a 400-B argument struct, event record without
// timing / system fence, stream wait on an event), per call, averaged over 2000 calls after warm-up.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
struct Big { char b[400]; };
__global__ void k_empty(Big a) { if (a.b[0] == 123 && threadIdx.x == 9999) a.b[1] = 0; }
int main() {
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
    Big a{};
    const int N = 2000;
    auto t = [&](const char* what, auto&& f) {
        for (int i = 0; i < 200; ++i) f();
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) f();
        auto t1 = std::chrono::steady_clock::now();
        hipDeviceSynchronize();
        printf("%-40s %7.2f us per call\n", what, std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    };
    t("kernel launch (400-B args)", [&] { k_empty<<<256, 256, 0, s1>>>(a); });
    t("event record", [&] { hipEventRecord(e, s1); });
    t("event record + wait on other stream", [&] { hipEventRecord(e, s1); hipStreamWaitEvent(s2, e, 0); });
    t("launch + record + wait", [&] { k_empty<<<256, 256, 0, s1>>>(a); hipEventRecord(e, s1); hipStreamWaitEvent(s2, e, 0); });
    t("hipMemsetAsync 4 KB", [&] { static void* p = nullptr; if (!p) hipMalloc(&p, 4096); hipMemsetAsync(p, 0, 4096, s1); });
    uint32_t* flag = nullptr;
    hipMalloc(&flag, 4096);
    hipMemset(flag, 0, 4096);
    uint32_t seq = 0;
    t("write value (stream 1)", [&] { hipStreamWriteValue32(s1, flag, ++seq, 0); });
    t("write value + wait value (>=) on stream 2", [&] {
        ++seq;
        hipStreamWriteValue32(s1, flag, seq, 0);
        hipStreamWaitValue32(s2, flag, seq, hipStreamWaitValueGte, 0xffffffffu);
    });
    t("launch + write + wait value", [&] {
        ++seq;
        k_empty<<<256, 256, 0, s1>>>(a);
        hipStreamWriteValue32(s1, flag, seq, 0);
        hipStreamWaitValue32(s2, flag, seq, hipStreamWaitValueGte, 0xffffffffu);
    });
    hipEvent_t e2;
    hipEventCreateWithFlags(&e2, hipEventDisableTiming);
    t("event record (fenced) + wait", [&] { hipEventRecord(e2, s1); hipStreamWaitEvent(s2, e2, 0); });
    t("wait only (event recorded once)", [&] { hipStreamWaitEvent(s2, e, 0); });
    // with the stream busy (the event not yet complete when the wait is enqueued)
    t("busy: launch + record (no fence) + wait", [&] { k_empty<<<256, 256, 0, s1>>>(a); hipEventRecord(e, s1); hipStreamWaitEvent(s2, e, 0); });
    t("busy: launch + record (fenced) + wait", [&] { k_empty<<<256, 256, 0, s1>>>(a); hipEventRecord(e2, s1); hipStreamWaitEvent(s2, e2, 0); });
    t("busy: launch only", [&] { k_empty<<<256, 256, 0, s1>>>(a); });
    t("busy: launch + write + wait value", [&] {
        ++seq;
        k_empty<<<256, 256, 0, s1>>>(a);
        hipStreamWriteValue32(s1, flag, seq, 0);
        hipStreamWaitValue32(s2, flag, seq, hipStreamWaitValueGte, 0xffffffffu);
    });
    return 0;
}
