// Wall time of the HIP set-up steps behind dbslmm_ctx_create (diagnostic probe of the CLI's
// end-to-end leg): runtime init, stream / event creation, kernel attribute calls (code object
// load), then the library's own dbslmm_ctx_create on a second context.
//   g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o tools/micro/hipinit tools/micro/hipinit.cpp \
//       -L dbslmm_amd -ldbslmm_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN/../../dbslmm_amd' -Wl,-rpath,/opt/rocm/lib
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include "../../include/dbslmm_hip.h"
extern "C" void dbslmm_chol_large();   // host stubs of kernels in libdbslmm_hip.so
extern "C" void dbslmm_gram_huge();
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    double t = now(), t0 = t;
    auto lap = [&](const char* what) { const double n = now(); printf("%-28s %.4f s\n", what, n - t); t = n; };
    int n = 0;
    (void)hipGetDeviceCount(&n); lap("hipGetDeviceCount");
    (void)hipSetDevice(0); lap("hipSetDevice");
    hipStream_t s[5];
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi); lap("getStreamPriorityRange");
    (void)hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking); lap("stream 1");
    (void)hipStreamCreateWithPriority(&s[1], hipStreamNonBlocking, hi); lap("stream 2 (high)");
    (void)hipStreamCreateWithPriority(&s[2], hipStreamNonBlocking, hi); lap("stream 3 (high)");
    (void)hipStreamCreateWithFlags(&s[3], hipStreamNonBlocking); lap("stream 4");
    (void)hipStreamCreateWithFlags(&s[4], hipStreamNonBlocking); lap("stream 5");
    hipEvent_t e;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming); lap("event");
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dbslmm_chol_large), hipFuncAttributeMaxDynamicSharedMemorySize, 65536); lap("first hipFuncSetAttribute");
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dbslmm_gram_huge), hipFuncAttributeMaxDynamicSharedMemorySize, 65536); lap("second hipFuncSetAttribute");
    void* d = nullptr;
    (void)hipMalloc(&d, 1 << 20); lap("hipMalloc 1 MiB");
    dbslmm_ctx* c = nullptr;
    const int rc = dbslmm_ctx_create(0, &c); lap("dbslmm_ctx_create (2nd ctx)");
    printf("total %.4f s rc=%d devices=%d\n", now() - t0, rc, n);
    return 0;
}
