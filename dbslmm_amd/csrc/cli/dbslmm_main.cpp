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
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
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
    string h2f;                     // "0.8,1,1.2": h2 factors of software/DBSLMM.R tuning
};

struct Allele { int64_t pos; string a1, a2; double maf; };                 // ALLELE
struct Summ { string snp; long ps; string a1, a2; double maf, z; };        // SUMM (P unused)
struct Info { string snp; long ps; int64_t pos; int block; string a1; double maf, z; };  // INFO

double walltime() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return static_cast<double>(tv.tv_sec) + tv.tv_usec * 1e-6;
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
    }
}

// IO::readBim (scr/dtpr.cpp:83-123): maf from the GPU MAF pass when constr.  Lines are split on
// several threads; the map keeps the first occurrence of a SNP id, as std::map::insert does.
bool read_bim(const string& ref, const vector<double>& maf, std::unordered_map<string, Allele>& bim,
              vector<string>& order) {
    const string text = read_file(ref + ".bim");
    if (text.empty()) { std::ifstream f(ref + ".bim"); return static_cast<bool>(f); }
    const vector<string_view> lines = lines_of(text);
    struct Row { string_view snp, a1, a2; bool ok; };
    vector<Row> rows(lines.size());
    parallel_chunks(lines.size(), host_threads(), [&](size_t lo, size_t hi) {
        vector<string_view> t;
        for (size_t i = lo; i < hi; ++i) {
            split_view(lines[i], '\t', t);
            rows[i] = t.size() < 6 ? Row{{}, {}, {}, false} : Row{t[1], t[4], t[5], true};
        }
    });
    bim.reserve(rows.size());
    for (size_t count = 0; count < rows.size(); ++count) {
        const Row& r = rows[count];
        if (!r.ok) continue;
        const double m = count < maf.size() ? maf[count] : 0.0;
        auto ins = bim.emplace(string(r.snp), Allele{static_cast<int64_t>(count), string(r.a1), string(r.a2), m});
        if (ins.second) order.push_back(ins.first->first);
    }
    return true;
}

// IO::readSumm (scr/dtpr.cpp:178-220): GEMMA, no header; z = beta/se when se starts with a digit
// and > 1e-20, else 0.  Parsed in contiguous line chunks on several threads, kept in file order.
vector<Summ> read_summ(const string& path) {
    const string text = read_file(path);
    const vector<string_view> lines = lines_of(text);
    vector<Summ> rows(lines.size());
    vector<char> ok(lines.size(), 0);
    parallel_chunks(lines.size(), host_threads(), [&](size_t lo, size_t hi) {
        vector<string_view> t;
        for (size_t i = lo; i < hi; ++i) {
            split_view(lines[i], '\t', t);
            if (t.size() < 11) continue;
            Summ& s = rows[i];
            s.z = 0.0;
            const string se_s(t[9]), b_s(t[8]), ps_s(t[2]), af_s(t[7]);
            if (isdigit(static_cast<unsigned char>(se_s.c_str()[0]))) {
                const double se = atof(se_s.c_str());
                if (se - 0.0 > 1e-20) s.z = atof(b_s.c_str()) / se;
            }
            s.snp = string(t[1]);
            s.ps = atol(ps_s.c_str());
            s.a1 = string(t[5]);
            s.a2 = string(t[6]);
            const double af = atof(af_s.c_str());
            s.maf = std::min(af, 1.0 - af);
            ok[i] = 1;
        }
    });
    vector<Summ> out;
    out.reserve(rows.size());
    for (size_t i = 0; i < rows.size(); ++i)
        if (ok[i]) out.push_back(std::move(rows[i]));
    return out;
}

struct Pos { string snp; long ps; int64_t pos; string a1; double maf, z; };

// SNPPROC::matchRef (scr/dtpr.cpp:383-408): strict allele equality, |maf_ref - maf| < mafMax.
// A SNP absent from the .bim compares against a default ALLELE ("", "", 0.0) as the reference's
// operator[] does, and is never kept.
vector<Pos> match_ref(const vector<Summ>& summ, const std::unordered_map<string, Allele>& bim,
                      double maf_max, vector<char>& good) {
    good.assign(summ.size(), 0);
    static const Allele empty{0, "", "", 0.0};
    const unsigned T = host_threads();
    vector<vector<Pos>> part(T);
    vector<int> dis_t(T, 0), maf_t(T, 0);
    vector<size_t> lo_t(T + 1, 0);
    for (unsigned t = 0; t <= T; ++t) lo_t[t] = summ.size() * t / T;
    vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (size_t i = lo_t[t]; i < lo_t[t + 1]; ++i) {
                auto it = bim.find(summ[i].snp);
                const Allele& b = it == bim.end() ? empty : it->second;
                const bool a1 = b.a1 == summ[i].a1, a2 = b.a2 == summ[i].a2;
                const bool mb = std::fabs(b.maf - summ[i].maf) < maf_max;
                if (!a1 || !a2) ++dis_t[t];
                if (!mb) ++maf_t[t];
                if (a1 && a2 && mb && it != bim.end()) {
                    part[t].push_back({summ[i].snp, summ[i].ps, b.pos, summ[i].a1, summ[i].maf, summ[i].z});
                    good[i] = 1;
                }
            }
        });
    for (auto& x : th) x.join();
    vector<Pos> inter;
    int dis = 0, mafc = 0;
    for (unsigned t = 0; t < T; ++t) {
        dis += dis_t[t];
        mafc += maf_t[t];
        for (auto& e : part[t]) inter.push_back(std::move(e));
    }
    std::cout << "Number of allele discrepency: " << dis << "\n";
    std::cout << "Number of maf discrepency:    " << mafc << "\n";
    return inter;
}

// SNPPROC::addBlock (scr/dtpr.cpp:455-481): [start, end), sequential scan; unassigned SNPs are
// dropped.
vector<Info> add_block(const vector<Pos>& inter, const vector<Block>& blocks) {
    vector<Info> out;
    size_t count = 0;
    for (size_t i = 0; i < blocks.size(); ++i) {
        for (size_t j = count; j < inter.size(); ++j) {
            if (inter[j].ps >= blocks[i].start && inter[j].ps < blocks[i].end) {
                out.push_back({inter[j].snp, inter[j].ps, inter[j].pos, static_cast<int>(i),
                               inter[j].a1, inter[j].maf, inter[j].z});
                ++count;
            } else {
                break;
            }
        }
    }
    return out;
}

void to_csr(const vector<Info>& info, int nb, vector<int64_t>& ptr, vector<int32_t>& pos, vector<double>& z) {
    ptr.assign(nb + 1, 0);
    for (const auto& e : info) ptr[e.block + 1]++;
    for (int b = 0; b < nb; ++b) ptr[b + 1] += ptr[b];
    pos.resize(info.size());
    z.resize(info.size());
    for (size_t i = 0; i < info.size(); ++i) {   // info is in block order (addBlock)
        pos[i] = static_cast<int32_t>(info[i].pos);
        z[i] = info[i].z;
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
bool align_test_pos(const vector<Info>& info, const vector<Info>& t_info, int nb, vector<int32_t>& out,
                    string& err) {
    vector<vector<int64_t>> per(nb);
    for (const auto& e : t_info) per[e.block].push_back(e.pos);
    vector<size_t> used(nb, 0);
    out.resize(info.size());
    for (size_t i = 0; i < info.size(); ++i) {
        const int b = info[i].block;
        if (used[b] >= per[b].size()) {
            err = "block " + std::to_string(b) + ": SNP " + info[i].snp + " has no counterpart in the test .bim";
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
    double t0 = walltime(), last = t0;
    string json;
    void mark(const char* name) {
        const double t = walltime();
        char buf[96];
        snprintf(buf, sizeof(buf), "%s\"%s\": %.6f", json.empty() ? "" : ", ", name, t - last);
        json += buf;
        last = t;
    }
    void print(int64_t n_snp) const {
        fprintf(stderr, "TIMING {%s, \"total\": %.6f, \"snps\": %lld}\n", json.c_str(), walltime() - t0,
                static_cast<long long>(n_snp));
    }
};

int main(int argc, char** argv) {
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

    std::cout << "Reading reference PLINK FAM file from [" << p.r << ".fam]\n";
    const int n_ref = get_row(p.r + ".fam");
    std::cout << n_ref << " individuals to be included from reference FAM file.\n";
    std::cout << "Reading reference PLINK BIM file from [" << p.r << ".bim]\n";
    const int n_snp_bim = get_row(p.r + ".bim");
    const bool constr = !(std::fabs(p.mafMax - 1.0) < 1e-10);

    dbslmm_ctx* ctx = nullptr;
    Mapped bed;
    if (!p.dry_run) {
        if (!bed.open(p.r + ".bed")) return fail(p.r + ".bed cannot be opened");
        if (p.gpu_ids.empty()) {
            if (dbslmm_ctx_create(p.gpu, &ctx) != DBSLMM_OK) return fail("no usable HIP device (dbslmm_ctx_create)");
            ph.mark("ctx");
            // one staged upload of the .bed serves both the MAF pass and the plan
            if (dbslmm_ctx_cache_bed(ctx, bed.p, static_cast<int64_t>(bed.n)) != DBSLMM_OK)
                return fail(string("uploading the .bed: ") + dbslmm_last_error(ctx));
            ph.mark("bed_upload");
        } else {
            vector<int32_t> ids;
            for (const string& t : split(p.gpu_ids, ',')) ids.push_back(atoi(t.c_str()));
            if (ids.empty() || dbslmm_ctx_create_multi(static_cast<int32_t>(ids.size()), ids.data(), &ctx) != DBSLMM_OK)
                return fail("no usable HIP devices (dbslmm_ctx_create_multi, --gpus / --gpu-ids)");
            std::cout << "Sharding the LD blocks over " << ids.size() << " GPUs.\n";
        }
    } else if (constr) {
        return fail("--dry-run needs -mafMax 1 (the MAF pass runs on the GPU)");
    }
    vector<double> maf;
    if (constr) {
        std::cout << "Calculating MAF of reference panel ...\n";
        maf.resize(n_snp_bim);
        if (dbslmm_bed_maf(ctx, bed.p, static_cast<int64_t>(bed.n), n_ref, n_snp_bim, maf.data()) != DBSLMM_OK)
            return fail(string("MAF pass: ") + dbslmm_last_error(ctx));
        ph.mark("maf");
    } else {
        std::cout << "[WARNING] Do not consider the difference between reference panel and summary data ...\n";
    }
    std::unordered_map<string, Allele> bim;
    vector<string> bim_order;
    read_bim(p.r, maf, bim, bim_order);
    std::cout << bim.size() << " SNPs to be included from reference BIM file.\n";
    const vector<Block> blocks = read_block(p.b);

    std::cout << "Reading summary data of small effect SNPs from [" << p.s << "]\n";
    const vector<Summ> summ_s = read_summ(p.s);
    vector<char> good_s;
    const vector<Pos> inter_s = match_ref(summ_s, bim, p.mafMax, good_s);
    std::cout << "After filtering, " << inter_s.size() << " small effect SNPs are selected.\n";
    const vector<Info> info_s = add_block(inter_s, blocks);
    std::ofstream bad(p.eff + ".badsnps");
    for (size_t i = 0; i < summ_s.size(); ++i)
        if (!good_s[i]) bad << summ_s[i].snp << " " << 0 << "\n";

    vector<Info> info_l;
    vector<Pos> inter_l;
    bool has_l = false;
    if (lf) {
        std::cout << "Reading summary data of large effect SNPs from [" << p.l << "]\n";
        const vector<Summ> summ_l = read_summ(p.l);
        vector<char> good_l;
        inter_l = match_ref(summ_l, bim, p.mafMax, good_l);
        if (!inter_l.empty()) {
            info_l = add_block(inter_l, blocks);
            std::cout << "After filtering, " << inter_l.size() << " large effect SNPs are selected.\n";
            has_l = true;
        } else {
            std::cout << "After filtering, no large effect SNP is selected.\n";
        }
        for (size_t i = 0; i < summ_l.size(); ++i)
            if (!good_l[i]) bad << summ_l[i].snp << " " << 1 << "\n";
    }
    bad.close();
    // test panel of the variance output (scr/dbslmm.cpp:264-320)
    const bool want_var = !p.dat_str.empty() && !p.test_indicator_file.empty();
    if (!want_var && (!p.dat_str.empty() || !p.test_indicator_file.empty()))
        std::cout << "[NOTE] variance.txt needs both -dat_str and -test_indicator_file; skipped.\n";
    vector<int32_t> ts_pos, tl_pos, indicator;
    if (want_var) {
        const vector<long> base = read_test_bim(p.dat_str + ".bim");
        string err;
        if (!align_test_pos(info_s, add_block(make_pos_for_test_bim(base, inter_s), blocks),
                            static_cast<int>(blocks.size()), ts_pos, err) ||
            (has_l && !align_test_pos(info_l, add_block(make_pos_for_test_bim(base, inter_l), blocks),
                                      static_cast<int>(blocks.size()), tl_pos, err)))
            return fail("test panel " + p.dat_str + ": " + err);
        indicator = read_indicator(p.test_indicator_file);
        if (indicator.empty()) return fail(p.test_indicator_file + " is empty or missing");
    }

    const int nb = static_cast<int>(blocks.size());
    vector<int64_t> s_ptr, l_ptr;
    vector<int32_t> s_pos, l_pos;
    vector<double> z_s, z_l;
    to_csr(info_s, nb, s_ptr, s_pos, z_s);
    if (has_l) to_csr(info_l, nb, l_ptr, l_pos, z_l);
    if (p.dry_run) {
        std::cout << "dry-run: blocks " << nb << " small " << info_s.size() << " large " << info_l.size() << "\n";
        return 0;
    }

    ph.mark("parse");
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
    dbslmm_plan_destroy(plan);
    std::cout << "Fitting time: " << walltime() - t0 << " seconds.\n";
    ph.mark("variance");

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
        // output writer (scr/dbslmm.cpp:353-364, 391-395): large rows first, then small rows;
        // ostream's default double format is printf %g at precision 6 (17 with --precise-out),
        // formatted in parallel chunks and written in order
        FILE* out = fopen((name + ".txt").c_str(), "wb");
        if (!out) return fail(name + ".txt cannot be written");
        const double* bs = beta_s.data() + static_cast<size_t>(f) * info_s.size();
        const double* bl = beta_l.data() + static_cast<size_t>(f) * info_l.size();
        const int prec = p.precise ? 17 : 6;
        auto emit = [&](const vector<Info>& info, const double* beta, int flag) {
            const unsigned T = host_threads();
            vector<string> buf(T);
            vector<std::thread> th;
            for (unsigned t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    const size_t lo = info.size() * t / T, hi = info.size() * (t + 1) / T;
                    string& o = buf[t];
                    o.reserve((hi - lo) * 48);
                    char num[64];
                    for (size_t i = lo; i < hi; ++i) {
                        const double noscl = beta[i] / std::sqrt(2 * info[i].maf * (1 - info[i].maf));
                        if (std::isinf(noscl)) continue;
                        o += info[i].snp;
                        o += ' ';
                        o += info[i].a1;
                        o += ' ';
                        o.append(num, static_cast<size_t>(snprintf(num, sizeof(num), "%.*g", prec, beta[i])));
                        o += ' ';
                        o.append(num, static_cast<size_t>(snprintf(num, sizeof(num), "%.*g", prec, noscl)));
                        o += flag ? " 1\n" : " 0\n";
                    }
                });
            for (auto& x : th) x.join();
            for (const string& o : buf) fwrite(o.data(), 1, o.size(), out);
        };
        emit(info_l, bl, 1);
        emit(info_s, bs, 0);
        fclose(out);
    }
    ph.mark("write");
    dbslmm_ctx_destroy(ctx);
    if (p.timing) ph.print(static_cast<int64_t>(info_s.size() + info_l.size()));
    return 0;
}
