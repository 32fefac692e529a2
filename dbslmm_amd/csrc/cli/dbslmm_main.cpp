// dbslmm_main.cpp -- drop-in `dbslmm` command line on top of libdbslmm_hip.so.
//
// Same flags, files and output formats as the reference binary (scr/main_dbslmm.cpp,
// scr/dbslmm.cpp:67-398).  The host steps (argument parsing, .fam/.bim/block/summary readers,
// allele + MAF matching, block assignment, output writers) are restated here in plain C++
// (reference: scr/dtpr.cpp:47-220, 383-481); the hot path -- the MAF pass of readBim and
// DBSLMMFIT::est -- goes through the C-ABI (include/dbslmm_hip.h) to the GPU.
//
// Extensions (not in the reference): --gpu N (HIP device), --gpus N (devices 0..N-1: the LD
// blocks sharded over N GPUs, dbslmm_ctx_create_multi), --gpu-ids a,b,.. (explicit device list,
// repeats allowed), --tau T (default 0.8 as hard-coded at
// scr/dbslmmfit.cpp:697,751), --precise-out (17 significant digits), --dry-run (stop after
// matching; prints counts, no GPU).  With -dat_str and -test_indicator_file the test-set variance
// matrix is written to ./variance.txt (arma_ascii, scr/dbslmmfit.cpp:242), evaluated on the GPU
// from the solve's factorisation (dbslmm_plan_variance); with -h2f it belongs to the last factor,
// as the reference's file after the driver's last run.
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <future>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../../include/dbslmm_hip.h"
#include "host_io.hpp"

using std::string;
using std::vector;

namespace {
using namespace dbslmm_host;

struct Param {                     // PARAM, scr/dbslmm.hpp:29-45 (initialised here)
    string s, l, r, b, eff, test_indicator_file, dat_str;
    int n = 0, nsnp = 0, t = 1;
    double mafMax = 1.0, h = -1.0;
    // extensions
    int gpu = 0;
    string gpu_ids;                 // --gpus N -> "0,1,..,N-1"; --gpu-ids a,b,..
    double tau = 0.8;
    bool precise = false, dry_run = false, h2f_merged = false, timing = false;
    int repeat = 0;                 // --repeat N: N more solves of the resident problem (timing)
    int parse_threads = 8;          // --parse-threads N: host parser threads beside the GPU set-up
    string h2f;                     // "0.8,1,1.2": h2 factors of software/DBSLMM.R tuning
};

// The host rows keep string_views into the mmap'd input files (no per-SNP allocation).
struct Bim {                        // map<string, ALLELE> of IO::readBim: line index = .bed row
    vector<string_view> snp, a1, a2;
    vector<char> bad;               // fewer than 6 fields: not inserted (the row still counts)
    vector<double> maf;             // GPU MAF pass (constr), else empty (0.0)
    StrIndex idx;                   // snp -> first line with it (std::map::insert keeps the first)
};
struct Summ { string_view snp, a1, a2; long ps; double maf, z; };         // SUMM (P unused)
struct Pos { int32_t summ; long ps; int64_t pos; };                       // POS: row of the summary
struct Info { int32_t summ; long ps; int64_t pos; int block; };           // INFO (fields via summ)

double walltime() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return static_cast<double>(tv.tv_sec) + tv.tv_usec * 1e-6;
}

// --timing: seconds from the process start (kernel start time, clock ticks) to now -- the loader
// and static initialisers before main
double since_process_start() {
    FILE* f = fopen("/proc/self/stat", "r");
    if (!f) return -1.0;
    char buf[1024];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    const char* q = strrchr(buf, ')');          // fields after the command name
    if (!q) return -1.0;
    unsigned long long start = 0;
    int field = 2;
    for (const char* c = q + 1; *c; ++c)
        if (*c == ' ' && ++field == 22) { start = strtoull(c + 1, nullptr, 10); break; }
    struct timespec ts;
    clock_gettime(CLOCK_BOOTTIME, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9 - static_cast<double>(start) / sysconf(_SC_CLK_TCK);
}

void print_header() {
    std::cout << "\n*************************************************************\n"
              << "  Deterministic Bayesian Sparse Linear Mixed Model (DBSLMM)  \n"
              << "  MI355X (gfx950) build of the per-LD-block solver          \n"
              << "  For Help, Type ./dbslmm -h                                 \n"
              << "*************************************************************\n\n";
}

void print_help() {
    std::cout << " FILE I/O RELATED OPTIONS\n"
              << " -s        [filename]   specify input the summary data for the small effect SNPs.\n"
              << " -l        [filename]   specify input the summary data for the large effect SNPs.\n"
              << " -r        [filename]   specify input the bfile of reference data.\n"
              << " -n        [num]        specify input the sample size of the summary data.\n"
              << " -mafMax   [num]        specify input the maximium of the difference between reference panel and summary data.\n"
              << " -nsnp     [num]   specify input the number of snp.\n"
              << " -b        [num]        specify input the block information.\n"
              << " -h        [num]        specify input the heritability.\n"
              << " -t        [filename]   specify input thread.\n"
              << " -eff      [filename]   specify output the estimate effect SNPs.\n"
              << " --gpu     [num]        HIP device (extension)\n"
              << " --gpus    [num]        shard the LD blocks over devices 0..num-1 (extension)\n"
              << " --gpu-ids [list]       shard over the listed devices, e.g. 0,1,2 (extension)\n"
              << " --tau     [num]        LD shrinkage, default 0.8 (extension)\n"
              << " --precise-out          17 significant digits in <eff>.txt (extension)\n"
              << " --timing               phase wall times as one JSON line on stderr (extension)\n"
              << " --parse-threads [num]  host parser threads while the GPU is set up (default 8; extension)\n"
              << " --repeat  [num]        with --timing: num more solves of the resident problem, their\n"
              << "                        wall times in the JSON line as solve_repeat (extension)\n"
              << " -h2f      [list]       h2 factors, e.g. 0.8,1,1.2: one Gram, one solve per factor,\n"
              << "                        <eff>_h2f<f>.txt each (software/DBSLMM.R tuning, extension)\n"
              << " --h2f-merged           -h2f: one factorisation per factor instead of one factor +\n"
              << "                        Chebyshev iteration for the big blocks (extension)\n";
}

// DBSLMM::Assign (scr/dbslmm.cpp:67-172): a flag's value is skipped when it starts with '-'.
void assign(int argc, char** argv, Param& p) {
    auto take = [&](int& i) -> const char* {
        if (i + 1 >= argc || argv[i + 1] == nullptr || argv[i + 1][0] == '-') return nullptr;
        return argv[++i];
    };
    for (int i = 0; i < argc; ++i) {
        const char* a = argv[i];
        const char* v = nullptr;
        auto is = [&](const char* x, const char* y) { return !strcmp(a, x) || !strcmp(a, y); };
        if (is("--smallEff", "-s")) { if ((v = take(i))) p.s = v; }
        else if (is("--largeEff", "-l")) { if ((v = take(i))) p.l = v; }
        else if (is("--reference", "-r")) { if ((v = take(i))) p.r = v; }
        else if (is("--N", "-n")) { if ((v = take(i))) p.n = atoi(v); }
        else if (is("--mafMax", "-mafMax")) { if ((v = take(i))) p.mafMax = atof(v); }
        else if (is("--numSNP", "-nsnp")) { if ((v = take(i))) p.nsnp = atoi(v); }
        else if (is("--block", "-b")) { if ((v = take(i))) p.b = v; }
        else if (is("--Heritability", "-h")) { if ((v = take(i))) p.h = atof(v); }
        else if (is("--Thread", "-t")) { if ((v = take(i))) p.t = atoi(v); }
        else if (is("--EFF", "-eff")) { if ((v = take(i))) p.eff = v; }
        else if (is("--test_indicator_file", "-test_indicator_file")) { if ((v = take(i))) p.test_indicator_file = v; }
        else if (is("--dat_str", "-dat_str")) { if ((v = take(i))) p.dat_str = v; }
        else if (!strcmp(a, "--gpu")) { if ((v = take(i))) p.gpu = atoi(v); }
        else if (!strcmp(a, "--gpus")) {
            if ((v = take(i))) {
                p.gpu_ids.clear();
                for (int g = 0; g < std::max(1, atoi(v)); ++g) p.gpu_ids += (g ? "," : "") + std::to_string(g);
            }
        }
        else if (!strcmp(a, "--gpu-ids")) { if ((v = take(i))) p.gpu_ids = v; }
        else if (!strcmp(a, "--tau")) { if ((v = take(i))) p.tau = atof(v); }
        else if (!strcmp(a, "--precise-out")) p.precise = true;
        else if (is("--h2f", "-h2f")) { if ((v = take(i))) p.h2f = v; }
        else if (!strcmp(a, "--h2f-merged")) p.h2f_merged = true;
        else if (!strcmp(a, "--dry-run")) p.dry_run = true;
        else if (!strcmp(a, "--timing")) p.timing = true;
        else if (!strcmp(a, "--repeat")) { if ((v = take(i))) p.repeat = std::max(0, atoi(v)); }
        else if (!strcmp(a, "--parse-threads")) { if ((v = take(i))) p.parse_threads = std::max(1, atoi(v)); }
    }
}

// IO::readBim (scr/dtpr.cpp:83-123): fields 1 (SNP), 4 (a1), 5 (a2) of each tab-separated line,
// parsed on several threads into views of the mapped file; the SNP index is built concurrently.
bool read_bim(const MappedText& f, Bim& bim) {
    if (!f.ok) return false;
    const unsigned T = host_threads();
    struct Row { string_view snp, a1, a2; bool ok; };
    vector<vector<Row>> part(T);
    const vector<size_t> cnt = parallel_lines(f.text, T, [&](unsigned t, string_view line) {
        string_view fl[6];
        part[t].push_back(tab_fields(line, fl, 6) < 6 ? Row{{}, {}, {}, false} : Row{fl[1], fl[4], fl[5], true});
    });
    size_t n = 0;
    for (size_t c : cnt) n += c;
    bim.snp.resize(n);
    bim.a1.resize(n);
    bim.a2.resize(n);
    bim.bad.assign(n, 0);
    vector<size_t> off(part.size() + 1, 0);
    for (size_t t = 0; t < part.size(); ++t) off[t + 1] = off[t] + part[t].size();
    parallel_chunks(part.size(), static_cast<unsigned>(part.size()), [&](size_t lo, size_t hi) {
        for (size_t t = lo; t < hi; ++t)
            for (size_t k = 0; k < part[t].size(); ++k) {
                const Row& r = part[t][k];
                const size_t i = off[t] + k;
                bim.snp[i] = r.snp;
                bim.a1[i] = r.a1;
                bim.a2[i] = r.a2;
                bim.bad[i] = !r.ok;
            }
    });
    bim.idx.build(n, T, [&](size_t i) { return bim.snp[i]; }, &bim.bad);
    return true;
}
size_t bim_size(const Bim& bim) {             // distinct SNP ids (std::map size)
    size_t n = 0;
    for (const auto& s : bim.idx.slot) n += s.load(std::memory_order_relaxed) >= 0;
    return n;
}

// IO::readSumm (scr/dtpr.cpp:178-220): GEMMA, no header; z = beta/se when se starts with a digit
// and > 1e-20, else 0.  Parsed in line chunks on several threads, kept in file order.
vector<Summ> read_summ(const MappedText& f) {
    const unsigned T = host_threads();
    vector<vector<Summ>> part(T);
    parallel_lines(f.text, T, [&](unsigned t, string_view line) {
        string_view fl[11];
        if (tab_fields(line, fl, 11) < 11) return;
        Summ s;
        s.z = 0.0;
        if (!fl[9].empty() && isdigit(static_cast<unsigned char>(fl[9][0]))) {
            const double se = field_atof(fl[9]);
            if (se - 0.0 > 1e-20) s.z = field_atof(fl[8]) / se;
        }
        s.snp = fl[1];
        s.ps = field_atol(fl[2]);
        s.a1 = fl[5];
        s.a2 = fl[6];
        const double af = field_atof(fl[7]);
        s.maf = std::min(af, 1.0 - af);
        part[t].push_back(s);
    });
    vector<Summ> out;
    size_t n = 0;
    for (const auto& v : part) n += v.size();
    out.reserve(n);
    for (const auto& v : part) out.insert(out.end(), v.begin(), v.end());
    return out;
}

// the .bim row of every summary SNP (-1: absent): the hashed half of matchRef, which needs no MAF,
// so it runs while the GPU thread still uploads the .bed and computes the MAF pass
vector<int32_t> lookup_ref(const vector<Summ>& summ, const Bim& bim) {
    vector<int32_t> row(summ.size());
    auto key = [&](size_t i) { return bim.snp[i]; };
    parallel_chunks(summ.size(), host_threads(), [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) row[i] = bim.idx.find(summ[i].snp, key);
    });
    return row;
}

// SNPPROC::matchRef (scr/dtpr.cpp:383-408): strict allele equality, |maf_ref - maf| < mafMax.
// A SNP absent from the .bim compares against a default ALLELE ("", "", 0.0) as the reference's
// operator[] does, and is never kept.
vector<Pos> match_ref(const vector<Summ>& summ, const Bim& bim, const vector<int32_t>& rows, double maf_max,
                      vector<char>& good) {
    good.assign(summ.size(), 0);
    const unsigned T = host_threads();
    vector<vector<Pos>> part(T);
    vector<int> dis_t(T, 0), maf_t(T, 0);
    vector<size_t> lo_t(T + 1, 0);
    for (unsigned t = 0; t <= T; ++t) lo_t[t] = summ.size() * t / T;
    vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (size_t i = lo_t[t]; i < lo_t[t + 1]; ++i) {
                const Summ& s = summ[i];
                const int32_t r = rows[i];
                const string_view b1 = r >= 0 ? bim.a1[r] : string_view(), b2 = r >= 0 ? bim.a2[r] : string_view();
                const double bm = r >= 0 && !bim.maf.empty() ? bim.maf[r] : 0.0;
                const bool a1 = b1 == s.a1, a2 = b2 == s.a2;
                const bool mb = std::fabs(bm - s.maf) < maf_max;
                if (!a1 || !a2) ++dis_t[t];
                if (!mb) ++maf_t[t];
                if (a1 && a2 && mb && r >= 0) {
                    part[t].push_back({static_cast<int32_t>(i), s.ps, static_cast<int64_t>(r)});
                    good[i] = 1;
                }
            }
        });
    for (auto& x : th) x.join();
    vector<Pos> inter;
    int dis = 0, mafc = 0;
    size_t n = 0;
    for (unsigned t = 0; t < T; ++t) n += part[t].size();
    inter.reserve(n);
    for (unsigned t = 0; t < T; ++t) {
        dis += dis_t[t];
        mafc += maf_t[t];
        inter.insert(inter.end(), part[t].begin(), part[t].end());
    }
    std::cout << "Number of allele discrepency: " << dis << "\n";
    std::cout << "Number of maf discrepency:    " << mafc << "\n";
    return inter;
}

// SNPPROC::addBlock (scr/dtpr.cpp:455-481): [start, end), sequential scan; unassigned SNPs are
// dropped.
vector<Info> add_block(const vector<Pos>& inter, const vector<Block>& blocks) {
    vector<Info> out;
    out.reserve(inter.size());
    size_t count = 0;
    for (size_t i = 0; i < blocks.size(); ++i) {
        for (size_t j = count; j < inter.size(); ++j) {
            if (inter[j].ps >= blocks[i].start && inter[j].ps < blocks[i].end) {
                out.push_back({inter[j].summ, inter[j].ps, inter[j].pos, static_cast<int>(i)});
                ++count;
            } else {
                break;
            }
        }
    }
    return out;
}

void to_csr(const vector<Info>& info, const vector<Summ>& summ, int nb, vector<int64_t>& ptr,
            vector<int32_t>& pos, vector<double>& z) {
    ptr.assign(nb + 1, 0);
    for (const auto& e : info) ptr[e.block + 1]++;
    for (int b = 0; b < nb; ++b) ptr[b + 1] += ptr[b];
    pos.resize(info.size());
    z.resize(info.size());
    for (size_t i = 0; i < info.size(); ++i) {   // info is in block order (addBlock)
        pos[i] = static_cast<int32_t>(info[i].pos);
        z[i] = summ[info[i].summ].z;
    }
}

// readTestBim (scr/calc_asymptotic_variance.cpp:142-153): the bp (4th tab field) of each line
vector<long> read_test_bim(const string& path) {
    vector<long> out;
    std::ifstream f(path);
    string line;
    while (std::getline(f, line)) {
        auto t = split(line, '\t');
        out.push_back(t.size() > 3 ? atol(t[3].c_str()) : 0);
    }
    return out;
}

// makePosObjectForTestBim (scr/calc_asymptotic_variance.cpp:160-180): pos = the FIRST test .bim
// line with the SNP's bp; SNPs without one are dropped
vector<Pos> make_pos_for_test_bim(const vector<long>& base, const vector<Pos>& inter) {
    std::unordered_map<long, int64_t> first;
    for (size_t i = 0; i < base.size(); ++i) first.emplace(base[i], static_cast<int64_t>(i));
    vector<Pos> out;
    for (const Pos& e : inter) {
        auto it = first.find(e.ps);
        if (it == first.end()) continue;
        Pos q = e;
        q.pos = it->second;
        out.push_back(q);
    }
    return out;
}

// read_indices_file (scr/subset_to_test_and_training.cpp:132-150): first space field per line
vector<int32_t> read_indicator(const string& path) {
    vector<int32_t> out;
    std::ifstream f(path);
    string line;
    while (std::getline(f, line)) out.push_back(static_cast<int32_t>(atol(split(line, ' ').empty() ? "0" : split(line, ' ')[0].c_str())));
    return out;
}

// calcBlock pairs the i-th SNP of a block with the i-th test SNP of the same block
// (test_info_s_block[i].pos, scr/dbslmmfit.cpp:394-396); a block with fewer test SNPs is an
// out-of-range read in the reference and an error here.
bool align_test_pos(const vector<Info>& info, const vector<Info>& t_info, const vector<Summ>& summ, int nb,
                    vector<int32_t>& out, string& err) {
    vector<vector<int64_t>> per(nb);
    for (const auto& e : t_info) per[e.block].push_back(e.pos);
    vector<size_t> used(nb, 0);
    out.resize(info.size());
    for (size_t i = 0; i < info.size(); ++i) {
        const int b = info[i].block;
        if (used[b] >= per[b].size()) {
            err = "block " + std::to_string(b) + ": SNP " + string(summ[info[i].summ].snp) +
                  " has no counterpart in the test .bim";
            return false;
        }
        out[i] = static_cast<int32_t>(per[b][used[b]++]);
    }
    return true;
}

// arma::Mat::save(..., arma_ascii) for a double matrix: header, dims, then each row with every
// element preceded by a space in scientific notation (precision 14, width 22)
bool save_arma_ascii(const string& path, const vector<double>& colmajor, int64_t rows, int64_t cols) {
    std::ofstream f(path);
    if (!f) return false;
    f << "ARMA_MAT_TXT_FN008\n" << rows << ' ' << cols << '\n';
    f.setf(std::ios::scientific);
    f.precision(14);
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t c = 0; c < cols; ++c) {
            const double v = colmajor[static_cast<size_t>(c) * rows + r];
            f.put(' ');
            f.width(22);
            if (std::isnan(v)) f << "nan";
            else if (std::isinf(v)) f << (v > 0 ? "inf" : "-inf");
            else f << v;
        }
        f.put('\n');
    }
    return static_cast<bool>(f);
}

int fail(const string& msg) {
    std::cerr << "ERROR: " << msg << std::endl;
    return 1;
}

}  // namespace

// --timing: wall time of each phase (seconds), printed as one JSON line on stderr at exit
struct Phases {
    double pre_main = since_process_start();
    double t0 = walltime(), last = t0;
    string json;
    void put(const char* name, double sec) {
        char buf[96];
        snprintf(buf, sizeof(buf), "%s\"%s\": %.6f", json.empty() ? "" : ", ", name, sec);
        json += buf;
    }
    void put_raw(const char* name, const string& v) {
        json += (json.empty() ? "\"" : ", \"") + string(name) + "\": " + v;
    }
    void mark(const char* name) {
        const double t = walltime();
        put(name, t - last);
        last = t;
    }
    void print(int64_t n_snp) const {
        fprintf(stderr, "TIMING {%s, \"total\": %.6f, \"snps\": %lld}\n", json.c_str(), walltime() - t0,
                static_cast<long long>(n_snp));
    }
};

namespace {
// getRow (scr/dtpr.cpp:71-80) of a mapped text: the number of getline lines
int64_t count_lines(string_view t) {
    std::atomic<int64_t> total{0};
    parallel_chunks(t.size(), host_threads(), [&](size_t lo, size_t hi) {
        int64_t n = 0;
        for (size_t i = lo; i < hi;) {
            const void* e = memchr(t.data() + i, '\n', hi - i);
            if (!e) break;
            ++n;
            i = static_cast<size_t>(static_cast<const char*>(e) - t.data()) + 1;
        }
        total += n;
    });
    return total + (!t.empty() && t.back() != '\n' ? 1 : 0);
}

// One <eff>.txt per h2f factor (scr/dbslmm.cpp:353-364, 391-395): large rows first, then small
// rows, "snp a1 beta beta_noscl flag"; ostream's default double format = printf %g at precision 6
// (17 with --precise-out), produced by std::to_chars (the same digits, ~3x faster than snprintf).
// All files and row chunks are formatted on the host threads, then written at their offsets.
// Returns -1 on success, else the index of the first file that could not be opened, written or
// closed; every output of the call is then removed (none is left truncated or partly written).
struct EffList { const vector<Info>* info; const vector<Summ>* summ; const double* beta; int flag; };
long write_eff_files(const vector<string>& names, const vector<std::array<EffList, 2>>& lists, int prec) {
    const unsigned T = host_threads();
    struct Task { size_t file; int list; size_t lo, hi; string out; };
    vector<Task> tasks;
    for (size_t f = 0; f < names.size(); ++f)
        for (int l = 0; l < 2; ++l) {
            const size_t n = lists[f][l].info->size();
            const size_t k = std::max<size_t>(1, std::min<size_t>(T, n / 2048 + 1));
            for (size_t c = 0; c < k; ++c) tasks.push_back({f, l, n * c / k, n * (c + 1) / k, {}});
        }
    std::atomic<size_t> next{0};
    auto fmt = [&] {
        char num[64];
        for (size_t t; (t = next.fetch_add(1)) < tasks.size();) {
            Task& k = tasks[t];
            const EffList& L = lists[k.file][k.list];
            string& o = k.out;
            o.reserve((k.hi - k.lo) * 56);
            for (size_t i = k.lo; i < k.hi; ++i) {
                const Summ& s = (*L.summ)[(*L.info)[i].summ];
                const double b = L.beta[i];
                const double noscl = b / std::sqrt(2 * s.maf * (1 - s.maf));
                if (std::isinf(noscl)) continue;
                o.append(s.snp.data(), s.snp.size());
                o += ' ';
                o.append(s.a1.data(), s.a1.size());
                o += ' ';
                o.append(num, std::to_chars(num, num + sizeof(num), b, std::chars_format::general, prec).ptr);
                o += ' ';
                o.append(num, std::to_chars(num, num + sizeof(num), noscl, std::chars_format::general, prec).ptr);
                o += L.flag ? " 1\n" : " 0\n";
            }
        }
    };
    {
        vector<std::thread> th;
        for (unsigned t = 1; t < T; ++t) th.emplace_back(fmt);
        fmt();
        for (auto& x : th) x.join();
    }
    vector<int> fd(names.size(), -1);
    vector<off_t> off(tasks.size(), 0);
    long bad = -1;                       // first file that failed
    for (size_t f = 0; f < names.size(); ++f) {
        fd[f] = ::open((names[f] + ".txt").c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd[f] < 0 && bad < 0) bad = static_cast<long>(f);
    }
    const bool ok = bad < 0;
    off_t pos = 0;
    for (size_t t = 0; t < tasks.size(); ++t) {
        if (t > 0 && tasks[t].file != tasks[t - 1].file) pos = 0;
        off[t] = pos;
        pos += static_cast<off_t>(tasks[t].out.size());
    }
    std::atomic<long> wbad{static_cast<long>(names.size())};   // smallest file index a write failed on
    if (ok) {
        next = 0;
        auto wr = [&] {
            for (size_t t; (t = next.fetch_add(1)) < tasks.size();) {
                const string& o = tasks[t].out;
                size_t done = 0;
                while (done < o.size()) {
                    const ssize_t w = pwrite(fd[tasks[t].file], o.data() + done, o.size() - done, off[t] + done);
                    if (w <= 0) {
                        long cur = wbad.load();
                        const long f = static_cast<long>(tasks[t].file);
                        while (f < cur && !wbad.compare_exchange_weak(cur, f)) {}
                        break;
                    }
                    done += static_cast<size_t>(w);
                }
            }
        };
        vector<std::thread> th;
        for (unsigned t = 1; t < std::min<unsigned>(T, 8); ++t) th.emplace_back(wr);
        wr();
        for (auto& x : th) x.join();
    }
    if (bad < 0 && wbad.load() < static_cast<long>(names.size())) bad = wbad.load();
    for (size_t f = 0; f < names.size(); ++f)
        if (fd[f] >= 0 && ::close(fd[f]) != 0 && bad < 0) bad = static_cast<long>(f);
    if (bad >= 0)
        for (size_t f = 0; f < names.size(); ++f)
            if (fd[f] >= 0) ::unlink((names[f] + ".txt").c_str());   // ours: opened (created) above
    return bad;
}
}  // namespace

int main(int argc, char** argv) {
    if (dbslmm_abi_version() != DBSLMM_ABI_VERSION) {   // a stale build against another library
        std::fprintf(stderr, "ERROR: libdbslmm_hip has ABI %d, this dbslmm was built for %d: rebuild it\n",
                     dbslmm_abi_version(), DBSLMM_ABI_VERSION);
        return 1;
    }
    Phases ph;
    if (argc <= 1) { print_header(); return 0; }
    if (argc == 2 && argv[1][0] == '-' && argv[1][1] == 'h') { print_help(); return 0; }
    Param p;
    assign(argc, argv, p);

    std::cout << "Options: \n-s:      " << p.s << "\n-l:      " << p.l << "\n-r:      " << p.r
              << "\n-nsnp:   " << p.nsnp << "\n-n:      " << p.n << "\n-mafMax: " << p.mafMax
              << "\n-b:      " << p.b << "\n-h:      " << p.h << "\n-t:      " << p.t
              << "\n-eff:    " << p.eff << "\n";
    // input checks of BatchRun (scr/dbslmm.cpp:195-227)
    if (p.s.empty()) return fail("-s is no parameter!");
    std::ifstream sf(p.s), lf(p.l), rf(p.r + ".fam"), bf(p.b);
    if (!bf) return fail(p.b + " dose not exist!");
    if (!sf) return fail(p.s + " dose not exist!");
    if (!rf) return fail(p.r + " dose not exist!");
    if (p.b.empty()) return fail("-b is no parameter!");
    if (p.r.empty()) return fail(p.r + " dose not exist!");
    if (p.h > 1 || p.h < 0) return fail("-h is not correct (0, 1)!");
    if (p.t > 100 || p.t < 1) return fail("-t is not correct (1, 100)!");
    if (p.eff.empty()) return fail("-eff is no parameter!");
    if (p.nsnp <= 0 || p.n <= 0) return fail("-n and -nsnp must be positive!");
    const bool has_lfile = static_cast<bool>(lf);
    sf.close();
    lf.close();
    rf.close();
    bf.close();

    // The GPU side runs on its own host thread from here on, while this one parses the text
    // inputs: HIP context (runtime and device initialisation), one staged upload of the .bed cached
    // on the context (it serves the MAF pass and the plan), then -- once this thread has counted
    // the .fam and .bim lines -- the MAF pass of readBim.
    const bool constr = !(std::fabs(p.mafMax - 1.0) < 1e-10);
    dbslmm_ctx* ctx = nullptr;
    Mapped bed;
    vector<double> maf;
    vector<int32_t> ids;
    string gpu_err;
    double t_ctx = 0.0, t_up = 0.0, t_maf = 0.0;
    std::promise<std::pair<int, int64_t>> dims;     // (n_ref, .bim lines) for the MAF pass
    std::future<std::pair<int, int64_t>> dims_f = dims.get_future();
    std::thread gpu;
    if (!p.dry_run) {
        if (!bed.open(p.r + ".bed")) return fail(p.r + ".bed cannot be opened");
        if (!p.gpu_ids.empty())
            for (const string& t : split(p.gpu_ids, ',')) ids.push_back(atoi(t.c_str()));
        gpu = std::thread([&] {
            double t = walltime();
            if (ids.empty()) {
                if (dbslmm_ctx_create(p.gpu, &ctx) != DBSLMM_OK) { gpu_err = "no usable HIP device (dbslmm_ctx_create)"; return; }
                t_ctx = walltime() - t;
                t = walltime();
                if (dbslmm_ctx_cache_bed_fd(ctx, bed.fd, static_cast<int64_t>(bed.n), bed.p) != DBSLMM_OK) {
                    gpu_err = string("uploading the .bed: ") + dbslmm_last_error(ctx);
                    return;
                }
                t_up = walltime() - t;
            } else {
                if (dbslmm_ctx_create_multi(static_cast<int32_t>(ids.size()), ids.data(), &ctx) != DBSLMM_OK) {
                    gpu_err = "no usable HIP devices (dbslmm_ctx_create_multi, --gpus / --gpu-ids)";
                    return;
                }
                t_ctx = walltime() - t;
            }
            const std::pair<int, int64_t> nd = dims_f.get();
            if (constr) {
                t = walltime();
                maf.resize(nd.second);
                if (dbslmm_bed_maf(ctx, bed.p, static_cast<int64_t>(bed.n), nd.first, nd.second, maf.data()) != DBSLMM_OK) {
                    gpu_err = string("MAF pass: ") + dbslmm_last_error(ctx);
                    return;
                }
                t_maf = walltime() - t;
            }
        });
    } else if (constr) {
        return fail("--dry-run needs -mafMax 1 (the MAF pass runs on the GPU)");
    }

    // the parsers run on fewer threads until the GPU thread's set-up is done: the HIP runtime's
    // initialisation and the .bed upload's pread pool are the critical path, not the parsing
    g_host_threads_cap = static_cast<unsigned>(p.parse_threads);
    std::cout << "Reading reference PLINK FAM file from [" << p.r << ".fam]\n";
    const int n_ref = get_row(p.r + ".fam");
    std::cout << n_ref << " individuals to be included from reference FAM file.\n";
    std::cout << "Reading reference PLINK BIM file from [" << p.r << ".bim]\n";
    MappedText bim_txt;
    bim_txt.open(p.r + ".bim");
    const int64_t n_snp_bim = count_lines(bim_txt.text);
    dims.set_value({n_ref, n_snp_bim});

    // host parsing (overlaps the GPU thread)
    Bim bim;
    read_bim(bim_txt, bim);
    const double t_bim = walltime() - ph.t0;
    const vector<Block> blocks = read_block(p.b);
    MappedText s_txt, l_txt;
    s_txt.open(p.s);
    const vector<Summ> summ_s = read_summ(s_txt);
    vector<Summ> summ_l;
    if (has_lfile) {
        l_txt.open(p.l);
        summ_l = read_summ(l_txt);
    }
    const vector<int32_t> rows_s = lookup_ref(summ_s, bim);
    const vector<int32_t> rows_l = has_lfile ? lookup_ref(summ_l, bim) : vector<int32_t>();
    const double t_parse = walltime() - ph.t0;
    if (gpu.joinable()) gpu.join();
    g_host_threads_cap = 16;
    if (!gpu_err.empty()) return fail(gpu_err);
    if (!ids.empty()) std::cout << "Sharding the LD blocks over " << ids.size() << " GPUs.\n";
    if (constr) std::cout << "Calculating MAF of reference panel ...\n";
    else std::cout << "[WARNING] Do not consider the difference between reference panel and summary data ...\n";
    bim.maf = std::move(maf);
    ph.put("pre_main", ph.pre_main);
    ph.put("ctx", t_ctx);
    ph.put("bed_upload", t_up);
    ph.put("maf", t_maf);
    ph.put("parse", t_parse);
    ph.put("parse_bim", t_bim);
    ph.mark("gpu_wait");      // wall time from the start to here (parse and GPU set-up overlap)
    std::cout << bim_size(bim) << " SNPs to be included from reference BIM file.\n";

    std::cout << "Reading summary data of small effect SNPs from [" << p.s << "]\n";
    vector<char> good_s;
    const vector<Pos> inter_s = match_ref(summ_s, bim, rows_s, p.mafMax, good_s);
    std::cout << "After filtering, " << inter_s.size() << " small effect SNPs are selected.\n";
    const vector<Info> info_s = add_block(inter_s, blocks);
    string badtxt;
    for (size_t i = 0; i < summ_s.size(); ++i)
        if (!good_s[i]) { badtxt.append(summ_s[i].snp.data(), summ_s[i].snp.size()); badtxt += " 0\n"; }

    vector<Info> info_l;
    vector<Pos> inter_l;
    bool has_l = false;
    if (has_lfile) {
        std::cout << "Reading summary data of large effect SNPs from [" << p.l << "]\n";
        vector<char> good_l;
        inter_l = match_ref(summ_l, bim, rows_l, p.mafMax, good_l);
        if (!inter_l.empty()) {
            info_l = add_block(inter_l, blocks);
            std::cout << "After filtering, " << inter_l.size() << " large effect SNPs are selected.\n";
            has_l = true;
        } else {
            std::cout << "After filtering, no large effect SNP is selected.\n";
        }
        for (size_t i = 0; i < summ_l.size(); ++i)
            if (!good_l[i]) { badtxt.append(summ_l[i].snp.data(), summ_l[i].snp.size()); badtxt += " 1\n"; }
    }
    {
        FILE* bad = fopen((p.eff + ".badsnps").c_str(), "wb");
        if (bad) {
            fwrite(badtxt.data(), 1, badtxt.size(), bad);
            fclose(bad);
        }
    }
    // test panel of the variance output (scr/dbslmm.cpp:264-320)
    const bool want_var = !p.dat_str.empty() && !p.test_indicator_file.empty();
    if (!want_var && (!p.dat_str.empty() || !p.test_indicator_file.empty()))
        std::cout << "[NOTE] variance.txt needs both -dat_str and -test_indicator_file; skipped.\n";
    vector<int32_t> ts_pos, tl_pos, indicator;
    if (want_var) {
        const vector<long> base = read_test_bim(p.dat_str + ".bim");
        string err;
        if (!align_test_pos(info_s, add_block(make_pos_for_test_bim(base, inter_s), blocks), summ_s,
                            static_cast<int>(blocks.size()), ts_pos, err) ||
            (has_l && !align_test_pos(info_l, add_block(make_pos_for_test_bim(base, inter_l), blocks), summ_l,
                                      static_cast<int>(blocks.size()), tl_pos, err)))
            return fail("test panel " + p.dat_str + ": " + err);
        indicator = read_indicator(p.test_indicator_file);
        if (indicator.empty()) return fail(p.test_indicator_file + " is empty or missing");
    }

    const int nb = static_cast<int>(blocks.size());
    vector<int64_t> s_ptr, l_ptr;
    vector<int32_t> s_pos, l_pos;
    vector<double> z_s, z_l;
    to_csr(info_s, summ_s, nb, s_ptr, s_pos, z_s);
    if (has_l) to_csr(info_l, summ_l, nb, l_ptr, l_pos, z_l);
    ph.mark("match");
    if (p.dry_run) {
        std::cout << "dry-run: blocks " << nb << " small " << info_s.size() << " large " << info_l.size() << "\n";
        if (p.timing) ph.print(static_cast<int64_t>(info_s.size() + info_l.size()));
        std::cout.flush();
        std::_Exit(0);
    }

    const double sigma_s = p.h / static_cast<double>(p.nsnp);                 // dbslmm.cpp:332
    dbslmm_problem prob{};
    prob.bed = bed.p;
    prob.bed_len = static_cast<int64_t>(bed.n);
    prob.n_ref = n_ref;
    prob.n_obs = p.n;
    prob.sigma_s = sigma_s;
    prob.tau = p.tau;
    prob.num_block = nb;
    prob.s_ptr = s_ptr.data();
    prob.s_pos = s_pos.data();
    prob.z_s = z_s.data();
    if (has_l) {
        prob.l_ptr = l_ptr.data();
        prob.l_pos = l_pos.data();
        prob.z_l = z_l.data();
    }
    dbslmm_options opts{};
    opts.h2f_mode = p.h2f_merged ? 1 : 0;
    prob.opts = &opts;
    // h2 factors (software/DBSLMM.R:204-219 runs dbslmm with -h h2 * hh for each hh); without
    // -h2f a single run with factor 1 and the plain <eff>.txt name
    vector<double> factors;
    if (!p.h2f.empty()) {
        for (const string& t : split(p.h2f, ',')) factors.push_back(atof(t.c_str()));
        for (double f : factors)
            if (!(f > 0) || p.h * f > 1) return fail("-h2f: h * factor must be in (0, 1]");
    } else {
        factors.push_back(1.0);
    }
    const int nf = static_cast<int>(factors.size());
    opts.shard_copies = nf;   // --gpus N: the shard plan may split the h2f copies of the largest blocks
    vector<double> sigmas(nf);
    for (int i = 0; i < nf; ++i) sigmas[i] = p.h * factors[i] / static_cast<double>(p.nsnp);
    vector<double> beta_s(static_cast<size_t>(nf) * info_s.size()), beta_l(static_cast<size_t>(nf) * info_l.size());
    vector<int32_t> status(static_cast<size_t>(nf) * std::max(nb, 1));
    std::cout << "Fitting model...\n";
    const double t0 = walltime();
    dbslmm_plan* plan = nullptr;
    int rc = dbslmm_plan_create(ctx, &prob, &plan);
    ph.mark("plan");
    if (rc == DBSLMM_OK) rc = dbslmm_plan_run_multi(plan, sigmas.data(), nf, beta_s.data(), beta_l.data(), status.data());
    ph.mark("solve");
    if (p.timing && p.repeat > 0 && rc == DBSLMM_OK) {   // the same solve again, inputs resident
        string rep;
        for (int k = 0; k < p.repeat && rc == DBSLMM_OK; ++k) {
            const double r0 = walltime();
            rc = dbslmm_plan_run_multi(plan, sigmas.data(), nf, beta_s.data(), beta_l.data(), status.data());
            char buf[32];
            snprintf(buf, sizeof(buf), "%s%.6f", k ? ", " : "", walltime() - r0);
            rep += buf;
        }
        ph.put_raw("solve_repeat", "[" + rep + "]");
        ph.last = walltime();
    }
    if (rc != DBSLMM_OK) {
        dbslmm_plan_destroy(plan);
        return fail(string("dbslmm_plan_run_multi: ") + dbslmm_last_error(ctx));
    }
    if (want_var) {
        Mapped tbed;
        if (!tbed.open(p.dat_str + ".bed")) {
            dbslmm_plan_destroy(plan);
            return fail(p.dat_str + ".bed cannot be opened");
        }
        int64_t n_test = 0;
        for (int32_t v : indicator) n_test += v != 0;
        vector<double> diags(static_cast<size_t>(n_test) * nb);
        dbslmm_test_panel tp{tbed.p, static_cast<int64_t>(tbed.n), static_cast<int32_t>(indicator.size()),
                             indicator.data(), ts_pos.data(), has_l ? tl_pos.data() : nullptr};
        rc = dbslmm_plan_variance(plan, &tp, diags.data(), nullptr);
        if (rc != DBSLMM_OK) {
            dbslmm_plan_destroy(plan);
            return fail(string("dbslmm_plan_variance: ") + dbslmm_last_error(ctx));
        }
        if (!save_arma_ascii("variance.txt", diags, n_test, nb)) {
            dbslmm_plan_destroy(plan);
            return fail("variance.txt cannot be written");
        }
    }
    // (no dbslmm_plan_destroy / dbslmm_ctx_destroy on the way out: the process ends with _Exit
    // below and the driver releases its device memory; freeing ~10 GB first only delays the exit)
    std::cout << "Fitting time: " << walltime() - t0 << " seconds.\n";
    ph.mark("variance");

    vector<string> names;
    vector<std::array<EffList, 2>> lists;
    for (int f = 0; f < nf; ++f) {
        int n_bad = 0;
        for (int b = 0; b < nb; ++b) {
            const int32_t st = status[static_cast<size_t>(f) * nb + b];
            if (st == DBSLMM_BLOCK_NOT_PD || st == DBSLMM_BLOCK_MONOMORPHIC) ++n_bad;
        }
        if (n_bad) std::cerr << "ERROR: Matrix is Singular! (" << n_bad << " LD blocks, beta = nan)\n";
        // output name: <eff>.txt, or with -h2f the driver's <prefix>_h2f<hh>.dbslmm.txt
        string name = p.eff;
        if (!p.h2f.empty()) {
            char hh[32];
            snprintf(hh, sizeof(hh), "%.15g", factors[f]);
            const string ext = ".dbslmm";
            if (name.size() > ext.size() && name.compare(name.size() - ext.size(), ext.size(), ext) == 0)
                name = name.substr(0, name.size() - ext.size()) + "_h2f" + hh + ext;
            else
                name += string("_h2f") + hh;
        }
        names.push_back(name);
        lists.push_back({EffList{&info_l, &summ_l, beta_l.data() + static_cast<size_t>(f) * info_l.size(), 1},
                         EffList{&info_s, &summ_s, beta_s.data() + static_cast<size_t>(f) * info_s.size(), 0}});
    }
    if (const long bad = write_eff_files(names, lists, p.precise ? 17 : 6); bad >= 0)
        return fail(names[static_cast<size_t>(bad)] + ".txt cannot be written");
    ph.mark("write");
    if (p.timing) {
        ph.print(static_cast<int64_t>(info_s.size() + info_l.size()));
        fprintf(stderr, "EXIT_AT %.6f\n", walltime());
    }
    // the parsed inputs (views of the mappings, hash index, host arrays) need no teardown
    std::cout.flush();
    fflush(stderr);
    std::_Exit(0);
}
