// host_io.hpp -- host-side readers shared by the drop-in CLIs (dbslmm, valid): restatements of
// the reference's IO helpers (scr/dtpr.cpp) that are not on the GPU path.
#pragma once
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

namespace dbslmm_host {
using std::string;
using std::string_view;
using std::vector;

struct Block { string chr; long start, end; };                              // BLOCK

// fields of a line separated by sep, as std::getline over a stringstream yields them (a trailing
// separator does not add an empty field)
inline void split_view(string_view line, char sep, vector<string_view>& out) {
    out.clear();
    size_t i = 0;
    while (i < line.size()) {
        const size_t j = line.find(sep, i);
        if (j == string_view::npos) { out.push_back(line.substr(i)); break; }
        out.push_back(line.substr(i, j - i));
        i = j + 1;
    }
}
inline vector<string> split(const string& line, char sep) {
    vector<string_view> v;
    split_view(line, sep, v);
    return vector<string>(v.begin(), v.end());
}

// whole file in memory ("" if it cannot be read)
inline string read_file(const string& path) {
    string s;
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return s;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n > 0) {
        s.resize(static_cast<size_t>(n));
        s.resize(fread(&s[0], 1, s.size(), f));
    }
    fclose(f);
    return s;
}

// the lines of a text (std::getline semantics: the last line may lack its '\n'; a '\r' stays)
inline vector<string_view> lines_of(string_view text) {
    vector<string_view> out;
    size_t i = 0;
    while (i < text.size()) {
        const char* e = static_cast<const char*>(memchr(text.data() + i, '\n', text.size() - i));
        const size_t j = e ? static_cast<size_t>(e - text.data()) : text.size();
        out.push_back(text.substr(i, j - i));
        i = j + 1;
    }
    return out;
}

// run f(lo, hi) over [0, n) in up to `threads` contiguous chunks (order-preserving parsers)
template <typename F>
inline void parallel_chunks(size_t n, unsigned threads, F f) {
    threads = std::max(1u, std::min<unsigned>(threads, static_cast<unsigned>(n / 4096 + 1)));
    if (threads == 1) { f(size_t(0), n); return; }
    vector<std::thread> th;
    for (unsigned t = 0; t < threads; ++t)
        th.emplace_back(f, n * t / threads, n * (t + 1) / threads);
    for (auto& x : th) x.join();
}
// worker threads of the host parsers / writer: at most 16 (the CPU share of one GPU on the box);
// the dbslmm CLI lowers the cap while its GPU thread initialises the device and uploads the .bed
inline unsigned g_host_threads_cap = 16;
inline unsigned host_threads() {
    return std::max(1u, std::min(g_host_threads_cap, std::thread::hardware_concurrency()));
}

// IO::getRow (scr/dtpr.cpp:71-80)
inline int get_row(const string& path) {
    return static_cast<int>(lines_of(read_file(path)).size());
}

// IO::readBlock (scr/dtpr.cpp:47-68)
inline vector<Block> read_block(const string& path) {
    vector<Block> out;
    std::ifstream f(path);
    string line;
    while (std::getline(f, line)) {
        auto t = split(line, '\t');
        if (t.size() < 3) continue;
        out.push_back({t[0], atol(t[1].c_str()), atol(t[2].c_str())});
    }
    return out;
}

// mmap'd .bed image
struct Mapped {
    const uint8_t* p = nullptr;
    size_t n = 0;
    int fd = -1;
    bool open(const string& path) {
        fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        if (fstat(fd, &st) != 0) return false;
        n = static_cast<size_t>(st.st_size);
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) return false;
        p = static_cast<const uint8_t*>(m);
        return true;
    }
    ~Mapped() {
        if (p) munmap(const_cast<uint8_t*>(p), n);
        if (fd >= 0) close(fd);
    }
};

// ---------------------------------------------------------------- fast text ingest (dbslmm CLI)
// A page-cached text file mapped read-only; the parsers keep string_views into it (no per-field
// allocation), so the mapping lives as long as the parsed rows.
struct MappedText {
    Mapped m;
    string_view text;
    bool ok = false;
    bool open(const string& path) {
        struct stat st;
        if (::stat(path.c_str(), &st) != 0) return false;
        ok = true;
        if (st.st_size == 0) return true;
        if (!m.open(path)) return ok = false;
        text = string_view(reinterpret_cast<const char*>(m.p), m.n);
        return true;
    }
};

// Lines of `text` on up to `threads` threads, in order: thread t owns the lines that START in its
// byte range and calls f(t, line) for each (std::getline semantics: the last line may lack its
// '\n').  Returns the number of lines each thread saw (their prefix sum gives global line numbers).
template <typename F>
inline vector<size_t> parallel_lines(string_view text, unsigned threads, F f) {
    const size_t n = text.size();
    threads = std::max(1u, std::min<unsigned>(threads, static_cast<unsigned>(n / (1 << 16) + 1)));
    vector<size_t> count(threads, 0);
    auto run = [&](unsigned t) {
        size_t lo = n * t / threads, hi = n * (t + 1) / threads;
        // the first line starting at or after lo (a line starts after a '\n', or at 0)
        if (lo > 0) {
            const void* e = memchr(text.data() + lo - 1, '\n', n - (lo - 1));
            lo = e ? static_cast<size_t>(static_cast<const char*>(e) - text.data()) + 1 : n;
        }
        size_t i = lo, c = 0;
        while (i < hi && i < n) {
            const void* e = memchr(text.data() + i, '\n', n - i);
            const size_t j = e ? static_cast<size_t>(static_cast<const char*>(e) - text.data()) : n;
            f(t, text.substr(i, j - i));
            ++c;
            i = j + 1;
        }
        count[t] = c;
    };
    vector<std::thread> th;
    for (unsigned t = 1; t < threads; ++t) th.emplace_back(run, t);
    run(0);
    for (auto& x : th) x.join();
    return count;
}

// the first k tab-separated fields of a line (fewer if the line has fewer); returns the count
inline int tab_fields(string_view line, string_view* out, int k) {
    int c = 0;
    size_t i = 0;
    while (c < k && i < line.size()) {
        const void* e = memchr(line.data() + i, '\t', line.size() - i);
        const size_t j = e ? static_cast<size_t>(static_cast<const char*>(e) - line.data()) : line.size();
        out[c++] = line.substr(i, j - i);
        i = j + 1;
    }
    return c;
}

// atof / atol of a field that is not NUL-terminated, with the C library's semantics (leading
// white space, sign, longest valid prefix, 0 when there is none): strtod / strtol on a copy
inline double field_atof(string_view s) {
    char buf[64];
    if (s.size() < sizeof(buf)) {
        memcpy(buf, s.data(), s.size());
        buf[s.size()] = 0;
        return strtod(buf, nullptr);
    }
    return strtod(string(s).c_str(), nullptr);
}
inline long field_atol(string_view s) {
    // fast path: plain decimal digits (bp positions)
    if (!s.empty() && s.size() < 19) {
        long v = 0;
        size_t i = 0;
        for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; ++i) v = v * 10 + (s[i] - '0');
        if (i == s.size() && i > 0) return v;
    }
    char buf[64];
    if (s.size() < sizeof(buf)) {
        memcpy(buf, s.data(), s.size());
        buf[s.size()] = 0;
        return strtol(buf, nullptr, 10);
    }
    return strtol(string(s).c_str(), nullptr, 10);
}

inline uint64_t hash_sv(string_view s) {          // FNV-1a, 64 bit
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h ^ (h >> 29);
}

// Open-addressing index of n keys (key(i) -> string_view), built on several threads: every slot
// holds the SMALLEST i among equal keys (std::map::insert keeps the first occurrence).  Slots only
// go from empty to full, so equal keys always meet in one slot whatever the interleaving.
struct StrIndex {
    vector<std::atomic<int32_t>> slot;
    vector<uint64_t> hash;
    size_t mask = 0;
    template <typename K>
    void build(size_t n, unsigned threads, K key, const vector<char>* skip = nullptr) {
        size_t cap = 16;
        while (cap < 2 * n + 16) cap <<= 1;
        mask = cap - 1;
        slot = vector<std::atomic<int32_t>>(cap);
        hash.assign(n, 0);
        parallel_chunks(cap, threads, [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; ++i) slot[i].store(-1, std::memory_order_relaxed);
        });
        parallel_chunks(n, threads, [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; ++i) {
                if (skip && (*skip)[i]) continue;
                const string_view k = key(i);
                const uint64_t h = hash_sv(k);
                hash[i] = h;
                size_t p = h & mask;
                const int32_t me = static_cast<int32_t>(i);
                for (;;) {
                    int32_t cur = slot[p].load(std::memory_order_acquire);
                    if (cur < 0) {
                        if (slot[p].compare_exchange_strong(cur, me, std::memory_order_acq_rel)) break;
                        // another key took the slot: re-examine it
                    }
                    if (cur >= 0) {
                        if (hash[cur] == h && key(cur) == k) {   // equal key: keep the smaller index
                            while (me < cur && !slot[p].compare_exchange_weak(cur, me, std::memory_order_acq_rel)) {
                            }
                            break;
                        }
                        p = (p + 1) & mask;
                    }
                }
            }
        });
    }
    // index of key k, or -1
    template <typename K>
    int32_t find(string_view k, K key) const {
        const uint64_t h = hash_sv(k);
        size_t p = h & mask;
        for (;;) {
            const int32_t cur = slot[p].load(std::memory_order_relaxed);
            if (cur < 0) return -1;
            if (hash[cur] == h && key(cur) == k) return cur;
            p = (p + 1) & mask;
        }
    }
};

}  // namespace dbslmm_host
