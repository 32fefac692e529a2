"""Host sanitizers (ASan + UBSan) over the host-side C/C++ code (CPU suite, no GPU):

* the drop-in `dbslmm` / `valid` CLIs built with -fsanitize=address,undefined
  (`make -C dbslmm_amd/csrc sanitize`): argument handling and the whole host pipeline --
  .fam/.bim/summary/block readers, allele + MAF matching, addBlock, CSR assembly, .badsnps
  writer -- through --dry-run (stops before the first GPU call);
* the CPU oracle (`make -C oracle sanitize`): a standalone driver over every oracle entry point
  on the reference's test_dat panel and a synthetic panel with missing calls and n % 4 = 3.

A sanitizer report aborts the program (-fno-sanitize-recover), so a zero exit code is the
check.  The GPU kernels themselves cannot be sanitized on this pool (no GPU ASan / XNACK)."""
import os
import subprocess

import pytest

from _common import BLOCKS_EUR1, GOLD, ROOT, TD
from test_cli import SUMM, REF, split_summary

BIN = os.path.join(ROOT, "dbslmm_amd", "bin")
ORACLE_SAN = os.path.join(ROOT, "oracle", "build", "sanitize_main")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _built(target_dir, target, path):
    if not os.access(path, os.X_OK):
        r = subprocess.run(["make", "-s", "-C", target_dir, target], capture_output=True, text=True,
                           timeout=600)
        if r.returncode != 0:
            if "asan" in r.stderr.lower() or "ubsan" in r.stderr.lower():
                pytest.skip(f"toolchain without the sanitizer runtimes: {r.stderr[-300:]}")
            pytest.fail(f"make {target} failed: {r.stderr[-2000:]}")
    return path


def _run(exe, args, cwd=None):
    return subprocess.run([exe] + args, capture_output=True, text=True, cwd=cwd, timeout=300, env=ENV)


def _clean(r):
    return "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr


@pytest.fixture(scope="module")
def cli_asan():
    return _built(os.path.join(ROOT, "dbslmm_amd", "csrc"), "sanitize", os.path.join(BIN, "dbslmm_asan"))


@pytest.fixture(scope="module")
def valid_asan():
    return _built(os.path.join(ROOT, "dbslmm_amd", "csrc"), "sanitize", os.path.join(BIN, "valid_asan"))


def test_cli_host_pipeline_under_asan_ubsan(cli_asan, tmp_path):
    s, l = split_summary(tmp_path)
    for extra in ([], ["-l", l], ["-l", l, "-mafMax", "0.2"]):
        r = _run(cli_asan, ["-s", s, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp", "996", "-h",
                            "0.5", "-eff", str(tmp_path / "o"), "--dry-run"] + extra)
        assert _clean(r), r.stderr[-3000:]
        if "-mafMax" in extra:   # the MAF pass needs the GPU: refused cleanly without one
            continue
        assert r.returncode == 0 and "dry-run: blocks" in r.stdout, r.stderr[-3000:]


@pytest.mark.parametrize("args", [
    [],
    ["-h"],
    ["-r", REF, "-b", BLOCKS_EUR1, "-h", "0.5", "-eff", "x"],
    ["-s", SUMM, "-r", REF, "-b", "/nonexistent", "-h", "0.5", "-eff", "x"],
    ["-s", SUMM, "-r", REF, "-b", BLOCKS_EUR1, "-h", "1.5", "-n", "10", "-nsnp", "10", "-eff", "x"],
    ["-s", SUMM, "-r", REF, "-b", BLOCKS_EUR1, "-h", "-0.5", "-n", "2400", "-nsnp", "996", "-eff", "x",
     "--dry-run"],
    ["-s", SUMM, "-r", REF, "-b", BLOCKS_EUR1, "-h", "0.5", "-h2f", "0.8,,x", "-n", "2400", "-nsnp",
     "996", "-eff", "x", "--dry-run"],
    ["-s"],
])
def test_cli_argument_handling_under_asan_ubsan(cli_asan, args, tmp_path):
    r = _run(cli_asan, args, cwd=str(tmp_path))
    assert _clean(r), r.stderr[-3000:]
    assert r.returncode in (0, 1), (r.returncode, r.stderr[-3000:])


@pytest.mark.parametrize("args", [
    [],
    ["-s", "x", "-r", REF, "-b", BLOCKS_EUR1, "-r2", "o"],
    ["-d", "/nonexistent", "-s", "/nonexistent", "-r", REF, "-b", BLOCKS_EUR1, "-r2", "o"],
])
def test_valid_argument_handling_under_asan_ubsan(valid_asan, args, tmp_path):
    r = _run(valid_asan, args, cwd=str(tmp_path))
    assert _clean(r), r.stderr[-3000:]
    assert r.returncode in (0, 1), (r.returncode, r.stderr[-3000:])


@pytest.mark.parametrize("bed,n_ref,n_snp", [
    (os.path.join(TD, "ref_chr1.bed"), 400, 723),
    (os.path.join(GOLD, "synth_small", "ref.bed"), 203, 600),
])
def test_oracle_under_asan_ubsan(bed, n_ref, n_snp):
    exe = _built(os.path.join(ROOT, "oracle"), "sanitize", ORACLE_SAN)
    r = _run(exe, [bed, str(n_ref), str(n_snp)])
    assert _clean(r), r.stderr[-3000:]
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stderr[-3000:]
