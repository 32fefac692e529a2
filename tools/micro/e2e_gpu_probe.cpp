// The device side of the dbslmm CLI's set-up, timed step by step (diagnostic probe, round 4):
// first HIP call, dbslmm_ctx_create, the .bed upload from its file descriptor, the MAF pass, a
// plan-sized allocation, and the process exit that follows (the parent times the whole process).
//   g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o tools/micro/e2e_gpu_probe \
//       tools/micro/e2e_gpu_probe.cpp -L dbslmm_amd -ldbslmm_hip -L/opt/rocm/lib -lamdhip64 \
//       -Wl,-rpath,'$ORIGIN/../../dbslmm_amd' -Wl,-rpath,/opt/rocm/lib
//   tools/micro/e2e_gpu_probe ref.bed n_ref n_snp [alloc_gib]
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/dbslmm_hip.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s ref.bed n_ref n_snp [alloc_gib]\n", argv[0]); return 2; }
    const double t0 = now();
    double t = t0;
    auto lap = [&](const char* what) { const double n = now(); printf("%-24s %8.4f s  (at %.4f)\n", what, n - t, n - t0); t = n; };
    const int n_ref = atoi(argv[2]);
    const long long n_snp = atoll(argv[3]);
    const double alloc_gib = argc > 4 ? atof(argv[4]) : 0.0;
    const int fd = open(argv[1], O_RDONLY);
    struct stat st;
    fstat(fd, &st);
    const size_t n = static_cast<size_t>(st.st_size);
    const uint8_t* p = static_cast<const uint8_t*>(mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0));
    lap("mmap");
    int nd = 0;
    (void)hipGetDeviceCount(&nd);
    lap("hipGetDeviceCount");
    dbslmm_ctx* ctx = nullptr;
    if (dbslmm_ctx_create(0, &ctx) != DBSLMM_OK) { printf("ctx_create failed\n"); return 1; }
    lap("dbslmm_ctx_create");
    if (dbslmm_ctx_cache_bed_fd(ctx, fd, static_cast<int64_t>(n), p) != DBSLMM_OK) { printf("upload failed\n"); return 1; }
    lap("cache_bed_fd");
    std::vector<double> maf(n_snp);
    if (dbslmm_bed_maf(ctx, p, static_cast<int64_t>(n), n_ref, n_snp, maf.data()) != DBSLMM_OK) { printf("maf failed\n"); return 1; }
    lap("bed_maf (1st)");
    if (dbslmm_bed_maf(ctx, p, static_cast<int64_t>(n), n_ref, n_snp, maf.data()) != DBSLMM_OK) { printf("maf failed\n"); return 1; }
    lap("bed_maf (2nd)");
    if (alloc_gib > 0) {
        void* d = nullptr;
        const size_t b = static_cast<size_t>(alloc_gib * (1 << 30));
        (void)hipMalloc(&d, b);
        lap("hipMalloc");
        (void)hipMemset(d, 0, b);
        (void)hipDeviceSynchronize();
        lap("memset + sync");
    }
    printf("exit at %.4f\n", now() - t0);
    fflush(stdout);
    std::_Exit(0);
}
