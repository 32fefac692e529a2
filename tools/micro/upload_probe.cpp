// Host -> device upload costs on the box (diagnostic): pinned allocation, pread from the page
// cache with T threads, DMA of pinned chunks.   upload_probe <file>
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <sys/mman.h>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
    double t = now();
    int n = 0;
    hipGetDeviceCount(&n);
    hipSetDevice(0);
    hipFree(nullptr);
    printf("init %.3f s\n", now() - t);
    const int fd = open(argv[1], O_RDONLY);
    struct stat sb;
    fstat(fd, &sb);
    const size_t N = sb.st_size, C = size_t(64) << 20;
    void* d;
    t = now();
    hipMalloc(&d, N);
    printf("hipMalloc %.1f MB %.3f s\n", N / 1e6, now() - t);
    std::vector<void*> st(3);
    t = now();
    for (auto& p : st) hipHostMalloc(&p, C, hipHostMallocDefault);
    printf("hipHostMalloc 3 x 64 MB %.3f s\n", now() - t);
    for (int T : {1, 4, 8, 16, 32}) {
        t = now();
        size_t done = 0;
        for (size_t off = 0; off < std::min(N, size_t(1) << 30); off += C) {
            const size_t len = std::min(C, N - off), part = (len + T - 1) / T;
            std::vector<std::thread> th;
            for (int i = 0; i < T; ++i)
                th.emplace_back([&, i] { size_t a = i * part, z = std::min(len, a + part); if (a < z) (void)pread(fd, (char*)st[0] + a, z - a, off + a); });
            for (auto& x : th) x.join();
            done += len;
        }
        printf("pread T=%2d: %.1f GB/s\n", T, done / (now() - t) / 1e9);
    }
    hipStream_t s;
    hipStreamCreate(&s);
    t = now();
    size_t done = 0;
    for (size_t off = 0; off + C <= N; off += C) { hipMemcpyAsync((char*)d + off, st[(off / C) % 3], C, hipMemcpyHostToDevice, s); done += C; }
    hipStreamSynchronize(s);
    printf("DMA pinned 64 MB chunks: %.1f GB/s\n", done / (now() - t) / 1e9);
    // the page-cached file mapped and registered with HIP: one DMA straight from the mapping
    t = now();
    void* mp = mmap(nullptr, N, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
    printf("mmap+populate %.3f s\n", now() - t);
    t = now();
    hipError_t e = hipHostRegister(mp, N, hipHostRegisterReadOnly);
    printf("hipHostRegister(ReadOnly) rc=%d %.3f s\n", (int)e, now() - t);
    if (e != hipSuccess) {
        t = now();
        e = hipHostRegister(mp, N, hipHostRegisterDefault);
        printf("hipHostRegister(Default) rc=%d %.3f s\n", (int)e, now() - t);
    }
    if (e == hipSuccess) {
        t = now();
        hipMemcpyAsync(d, mp, N, hipMemcpyHostToDevice, s);
        hipStreamSynchronize(s);
        printf("DMA from registered mapping: %.1f GB/s\n", N / (now() - t) / 1e9);
        t = now();
        hipHostUnregister(mp);
        printf("hipHostUnregister %.3f s\n", now() - t);
    }
    // anonymous memory filled by T threads from the page cache, then registered
    t = now();
    char* am = static_cast<char*>(mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
    printf("anon mmap+populate %.3f s\n", now() - t);
    {
        t = now();
        const int T = 16;
        const size_t part = (N + T - 1) / T;
        std::vector<std::thread> th;
        for (int i = 0; i < T; ++i)
            th.emplace_back([&, i] { size_t a = i * part, z = std::min(N, a + part); size_t g = a; while (g < z) { ssize_t r = pread(fd, am + g, z - g, g); if (r <= 0) break; g += r; } });
        for (auto& x : th) x.join();
        printf("pread 16 thr into anon: %.1f GB/s\n", N / (now() - t) / 1e9);
    }
    t = now();
    e = hipHostRegister(am, N, hipHostRegisterDefault);
    printf("hipHostRegister(anon) rc=%d %.3f s\n", (int)e, now() - t);
    if (e == hipSuccess) {
        t = now();
        hipMemcpyAsync(d, am, N, hipMemcpyHostToDevice, s);
        hipStreamSynchronize(s);
        printf("DMA from registered anon: %.1f GB/s\n", N / (now() - t) / 1e9);
    }
    return 0;
}
