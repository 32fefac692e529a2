// valid_main.cpp -- drop-in `valid` command line (external-validation R^2 terms) on top of
// libdbslmm_hip.so.  Same flags, inputs and <r2>.txt output as the reference (scr/main_valid.cpp,
// scr/validate.cpp:55-262).  Host steps -- readDBSLMM, readExt, matchSumm, readBim (+ the MAF pass
// on the GPU), matchAll, the sequential block scan -- are restated here (scr/dtpr.cpp:125-166,
// 223-268, 411-455); the per-block products go through dbslmm_valid_blocks (GPU).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <map>
#include <unordered_map>

#include "../../../include/dbslmm_hip.h"
#include "host_io.hpp"

using namespace dbslmm_host;

namespace {

struct Param { string d, s, r, b, r2; double mafMax = 1.0; int gpu = 0; };          // PARAM
struct SummS { string snp, a1; double maf = 0.0, z = 0.0; };                           // SUMMS
struct SummC { string snp, a1; double maf, z1, z2; };                                   // SUMMC
struct SummP { string snp; double z1, z2; long pos, ps; };                              // SUMMP
struct AlleleB { long pos = 0, ps = 0; string a1, a2; double maf = 0.0; };              // ALLELEB

int fail(const string& msg) {
    std::cerr << "ERROR: " << msg << std::endl;
    return 1;
}

// VALID::Assign (scr/validate.cpp:68-120): a value starting with '-' is skipped
void assign(int argc, char** argv, Param& p) {
    auto take = [&](int& i) -> const char* {
        if (i + 1 >= argc || argv[i + 1] == nullptr || argv[i + 1][0] == '-') return nullptr;
        return argv[++i];
    };
    for (int i = 0; i < argc; ++i) {
        const char* a = argv[i];
        const char* v = nullptr;
        auto is = [&](const char* x, const char* y) { return !strcmp(a, x) || !strcmp(a, y); };
        if (is("--dbslmm", "-d")) { if ((v = take(i))) p.d = v; }
        else if (is("--summ", "-s")) { if ((v = take(i))) p.s = v; }
        else if (is("--reference", "-r")) { if ((v = take(i))) p.r = v; }
        else if (is("--mafMax", "-mafMax")) { if ((v = take(i))) p.mafMax = atof(v); }
        else if (is("--block", "-b")) { if ((v = take(i))) p.b = v; }
        else if (is("--R2", "-r2")) { if ((v = take(i))) p.r2 = v; }
        else if (!strcmp(a, "--gpu")) { if ((v = take(i))) p.gpu = atoi(v); }
    }
}

// IO::readDBSLMM (scr/dtpr.cpp:223-245): space separated, z = third column
vector<SummS> read_dbslmm(const string& path) {
    vector<SummS> out;
    std::ifstream f(path);
    string line;
    while (std::getline(f, line)) {
        auto t = split(line, ' ');
        SummS s;
        if (t.size() > 0) s.snp = t[0];
        if (t.size() > 1) s.a1 = t[1];
        if (t.size() > 2) s.z = atof(t[2].c_str());
        out.push_back(s);
    }
    return out;
}

// IO::readExt (scr/dtpr.cpp:248-268): space separated snp a1 maf z; std::map keeps the first
std::unordered_map<string, SummS> read_ext(const string& path) {
    std::unordered_map<string, SummS> out;
    std::ifstream f(path);
    string line;
    while (std::getline(f, line)) {
        auto t = split(line, ' ');
        if (t.size() < 4) continue;
        out.emplace(t[0], SummS{t[0], t[1], atof(t[2].c_str()), atof(t[3].c_str())});
    }
    return out;
}

}  // namespace

int main(int argc, char** argv) {
    if (dbslmm_abi_version() != DBSLMM_ABI_VERSION) {   // a stale build against another library
        std::cerr << "ERROR: libdbslmm_hip has ABI " << dbslmm_abi_version() << ", this valid was built for "
                  << DBSLMM_ABI_VERSION << ": rebuild it\n";
        return 1;
    }
    if (argc <= 1) {
        std::cout << "\n*************************************************************\n"
                  << "  Deterministic Bayesian Sparse Linear Mixed Model (DBSLMM)  \n"
                  << "  valid -- MI355X (gfx950) build                           \n"
                  << "  For Help, Type ./valid -h                                  \n"
                  << "*************************************************************\n\n";
        return 0;
    }
    if (argc == 2 && argv[1][0] == '-' && argv[1][1] == 'h') {
        std::cout << " FILE I/O RELATED OPTIONS\n"
                  << " -d        [filename]   specify input the result of DBSLMM.\n"
                  << " -s        [filename]   specify input the external summary data.\n"
                  << " -r        [filename]   specify input the bfile of reference data.\n"
                  << " -mafMax   [num]        specify input the maximium of the difference between reference panel and external data.\n"
                  << " -b        [filename]   specify input the block information.\n"
                  << " -r2       [num]        specify output r2.\n"
                  << " --gpu     [num]        HIP device (extension)\n";
        return 0;
    }
    Param p;
    assign(argc, argv, p);
    std::cout << "Options: \n-d:      " << p.d << "\n-s:      " << p.s << "\n-r:      " << p.r
              << "\n-mafMax: " << p.mafMax << "\n-b:      " << p.b << "\n-r2:      " << p.r2 << "\n";
    // input checks of VALID::BatchRun (scr/validate.cpp:141-180)
    std::ifstream dS(p.d), sS(p.s), rS(p.r + ".fam"), bS(p.b);
    if (p.d.empty()) return fail("-d is no parameter!");
    if (p.s.empty()) return fail("-s is no parameter!");
    if (p.r.empty()) return fail("-r is no parameter!");
    if (!dS) return fail(p.d + " dose not exist!");
    if (!sS) return fail(p.s + " dose not exist!");
    if (!rS) return fail(p.r + " dose not exist!");
    if (!bS) return fail(p.b + " dose not exist!");

    const int n_ref = get_row(p.r + ".fam");
    std::cout << n_ref << " individuals to be included from reference FAM file.\n";
    const vector<SummS> dbslmm = read_dbslmm(p.d);
    std::cout << dbslmm.size() << " SNPs in DBSLMM result. \n";
    const auto ext = read_ext(p.s);
    std::cout << ext.size() << " SNPs in external result. \n";
    // SNPPROC::matchSumm (scr/dtpr.cpp:411-433)
    vector<SummC> comb;
    int dis = 0;
    for (const SummS& s : dbslmm) {
        auto it = ext.find(s.snp);
        if (it == ext.end()) continue;
        const bool same = it->second.a1 == s.a1;
        if (!same) ++dis;
        comb.push_back({it->second.snp, s.a1, it->second.maf, s.z, same ? it->second.z : -it->second.z});
    }
    std::cout << "Number of allele discrepency: " << dis << "\n";
    std::cout << comb.size() << " SNPs are intersection of DBSLMM and external summary statistics. \n";

    // IO::readBim, ALLELEB overload (scr/dtpr.cpp:125-166), MAF pass on the GPU when constr
    const bool constr = !(std::fabs(p.mafMax - 1.0) < 1e-10);
    const int n_snp = get_row(p.r + ".bim");
    Mapped bed;
    if (!bed.open(p.r + ".bed")) return fail(p.r + ".bed cannot be opened");
    dbslmm_ctx* ctx = nullptr;
    if (dbslmm_ctx_create(p.gpu, &ctx) != DBSLMM_OK) return fail("no usable HIP device (dbslmm_ctx_create)");
    vector<double> maf(n_snp, 0.0);
    if (constr) {
        std::cout << "Calculating MAF of reference panel ...\n";
        if (dbslmm_bed_maf(ctx, bed.p, static_cast<int64_t>(bed.n), n_ref, n_snp, maf.data()) != DBSLMM_OK)
            return fail(string("MAF pass: ") + dbslmm_last_error(ctx));
    } else {
        std::cout << "[WARNING] Do not consider the difference between reference panel and external summary data ...\n";
    }
    std::unordered_map<string, AlleleB> bim;
    {
        std::ifstream f(p.r + ".bim");
        string line;
        long count = 0;
        while (std::getline(f, line)) {
            auto t = split(line, '\t');
            if (t.size() >= 6 && bim.find(t[1]) == bim.end())
                bim.emplace(t[1], AlleleB{count, atoi(t[3].c_str()), t[4], t[5], maf[count]});
            ++count;
        }
    }
    std::cout << bim.size() << " SNPs to be included from reference BIM file.\n";
    // SNPPROC::matchAll (scr/dtpr.cpp:436-455): bim A1 equal, |maf_ref - maf_ext| < mafMax, sort by bp
    vector<SummP> summp;
    for (const SummC& c : comb) {
        auto it = bim.find(c.snp);
        if (it == bim.end()) continue;
        if (it->second.a1 == c.a1 && std::fabs(it->second.maf - c.maf) < p.mafMax)
            summp.push_back({c.snp, c.z1, c.z2, it->second.pos, it->second.ps});
    }
    std::stable_sort(summp.begin(), summp.end(), [](const SummP& a, const SummP& b) { return a.ps < b.ps; });
    std::cout << summp.size() << " SNPs intersect.\n";
    const vector<Block> blocks = read_block(p.b);
    const int nb = static_cast<int>(blocks.size());
    std::cout << nb << " blocks for the chromesome.\n";
    // the sequential block scan of scr/validate.cpp:226-253 (stalls like addBlock)
    vector<int64_t> ptr(nb + 1, 0);
    vector<int32_t> pos;
    vector<double> z1, z2;
    size_t count = 0;
    for (int b = 0; b < nb; ++b) {
        for (size_t j = count; j < summp.size(); ++j) {
            if (summp[j].ps >= blocks[b].start && summp[j].ps < blocks[b].end) {
                pos.push_back(static_cast<int32_t>(summp[j].pos));
                z1.push_back(summp[j].z1);
                z2.push_back(summp[j].z2);
                ++count;
            } else {
                break;
            }
        }
        ptr[b + 1] = static_cast<int64_t>(pos.size());
    }
    vector<double> nume(nb), deno(nb);
    if (dbslmm_valid_blocks(ctx, bed.p, static_cast<int64_t>(bed.n), n_ref, nb, ptr.data(), pos.data(),
                            z1.data(), z2.data(), nume.data(), deno.data()) != DBSLMM_OK)
        return fail(string("dbslmm_valid_blocks: ") + dbslmm_last_error(ctx));
    std::ofstream out(p.r2 + ".txt");
    for (int b = 0; b < nb; ++b) out << nume[b] << " " << deno[b] << "\n";
    dbslmm_ctx_destroy(ctx);
    return 0;
}
