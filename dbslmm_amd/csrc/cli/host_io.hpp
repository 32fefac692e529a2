// host_io.hpp -- host-side readers shared by the drop-in CLIs (dbslmm, valid): restatements of
// the reference's IO helpers (scr/dtpr.cpp) that are not on the GPU path.
#pragma once
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
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
inline unsigned host_threads() {
    return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
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

}  // namespace dbslmm_host
