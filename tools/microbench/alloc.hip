// Host cost of stream-ordered allocation (hipMallocAsync/hipFreeAsync) vs size, pool release
// threshold = max (what fhs_context uses), and of hipMalloc/hipFree, on MI355X.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>
int main() {
    hipStream_t st;
    hipStreamCreate(&st);
    hipMemPool_t pool;
    hipDeviceGetDefaultMemPool(&pool, 0);
    uint64_t thr = UINT64_MAX;
    hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    auto now = [] { return std::chrono::steady_clock::now(); };
    for (size_t mb : {4, 64, 512, 4096}) {
        const size_t bytes = mb << 20;
        for (int rep = 0; rep < 3; ++rep) {
            void* p = nullptr;
            auto t0 = now();
            hipMallocAsync(&p, bytes, st);
            auto t1 = now();
            hipFreeAsync(p, st);
            auto t2 = now();
            hipStreamSynchronize(st);
            printf("async %5zu MB: malloc %8.3f ms free %8.3f ms\n", mb,
                   std::chrono::duration<double, std::milli>(t1 - t0).count(),
                   std::chrono::duration<double, std::milli>(t2 - t1).count());
        }
        // many small allocations of this total size, 4.7 MB each (one cfg2 plaintext)
        if (mb == 4096) {
            std::vector<void*> v(870);
            for (int rep = 0; rep < 2; ++rep) {
                auto t0 = now();
                for (auto& q : v) hipMallocAsync(&q, 4718592, st);
                auto t1 = now();
                for (auto& q : v) hipFreeAsync(q, st);
                auto t2 = now();
                hipStreamSynchronize(st);
                printf("async 870 x 4.5 MB: malloc %8.3f ms free %8.3f ms\n",
                       std::chrono::duration<double, std::milli>(t1 - t0).count(),
                       std::chrono::duration<double, std::milli>(t2 - t1).count());
            }
        }
        void* p = nullptr;
        auto t0 = now();
        hipMalloc(&p, bytes);
        auto t1 = now();
        hipFree(p);
        auto t2 = now();
        printf("sync  %5zu MB: malloc %8.3f ms free %8.3f ms\n", mb,
               std::chrono::duration<double, std::milli>(t1 - t0).count(),
               std::chrono::duration<double, std::milli>(t2 - t1).count());
    }
    return 0;
}
