// host_io.hpp -- host-side readers shared by the drop-in CLIs (dbslmm, valid): restatements of
// the reference's IO helpers (scr/dtpr.cpp) that are not on the GPU path.
#pragma once
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>

#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace dbslmm_host {
using std::string;
using std::vector;

struct Block { string chr; long start, end; };                              // BLOCK

inline vector<string> split(const string& line, char sep) {
    vector<string> out;
    string e;
    std::stringstream ss(line);
    while (std::getline(ss, e, sep)) out.push_back(e);
    return out;
}

// IO::getRow (scr/dtpr.cpp:71-80)
inline int get_row(const string& path) {
    std::ifstream f(path);
    string line;
    int n = 0;
    while (std::getline(f, line)) ++n;
    return n;
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
