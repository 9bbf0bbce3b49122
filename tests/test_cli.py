"""The drop-in CLI surface: the nine bin_* programs keep the reference's argv
contract, stdout report and CSV schema, and every variant's
filtered output is bit-exact with the serial reference semantics."""
import csv
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "digital_signal_processsing_amd", "cli")
sys.path.insert(0, CLI)
import run_benchmarks as rb  # noqa: E402

GPU_BINS = ["bin_parallel", "bin_shared", "bin_vec2", "bin_vec4", "bin_hillis", "bin_vhillis",
            "bin_blelloch", "bin_vblelloch"]
CSV_NAMES = {"bin_cpu": "SingleThreadCpu", "bin_parallel": "Parallel Averager",
             "bin_shared": "SM Parallel Averager", "bin_vec2": "Vectorized SM Parallel Averager",
             "bin_vec4": "Vectorized SM4 Parallel", "bin_hillis": "HillisSteele",
             "bin_vhillis": "Vectorized HillisSteele", "bin_blelloch": "Blelloch",
             "bin_vblelloch": "Vectorized Blelloch"}
HEADER = ("Algorithm,MemoryMode,N_Samples,Grade,BlockSize,H2D_ms,Compute_ms,D2H_ms,Total_ms,Init_ms,"
          "ColdStart_Total_ms,Bandwidth_GBs,Throughput_MSs,ColdStart_MSs").split(",")


def _bin(name):
    p = os.path.join(CLI, name)
    if not os.path.exists(p):
        subprocess.run(["make", "-s", "-j8", "-C", CLI], check=True)
    return p


def _run(name, *args, cwd):
    return subprocess.run([_bin(name), *map(str, args)], cwd=cwd, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, universal_newlines=True, timeout=600)


@pytest.fixture
def stereo_wav(tmp_path):
    rng = np.random.default_rng(7)
    data = rng.integers(-32768, 32767, size=(6001, 2), dtype=np.int16)
    path = tmp_path / "in.wav"
    rb.write_wav(str(path), data)
    return path, data


@pytest.mark.parametrize("args", [[], ["x.wav"], ["x.wav", "3"]])
def test_usage_error_exits_1(tmp_path, args):
    r = _run("bin_cpu", *args, cwd=tmp_path)
    assert r.returncode == 1 and "Usage" in r.stderr


@pytest.mark.parametrize("block", [0, 16, 33, 2048, "x"])
def test_block_size_validation(tmp_path, stereo_wav, block):
    r = _run("bin_cpu", stereo_wav[0], 3, block, cwd=tmp_path)
    assert r.returncode == 1


def test_bad_grade_and_missing_file_exit_nonzero(tmp_path, stereo_wav):
    assert _run("bin_cpu", stereo_wav[0], 0, 256, cwd=tmp_path).returncode == 1
    r = _run("bin_cpu", tmp_path / "missing.wav", 3, 256, cwd=tmp_path)
    assert r.returncode == 1 and "could not open file" in r.stdout   # reference exits 0 here


def test_wav_rejects_non_16bit(tmp_path):
    p = tmp_path / "u8.wav"
    raw = bytearray(open(_write_tmp(tmp_path), "rb").read())
    raw[34:36] = (8).to_bytes(2, "little")
    p.write_bytes(bytes(raw))
    r = _run("bin_cpu", p, 3, 256, cwd=tmp_path)
    assert r.returncode == 1 and "unsupported bits per sample" in r.stdout


def _write_tmp(tmp_path):
    p = tmp_path / "small.wav"
    rb.write_wav(str(p), np.arange(20, dtype=np.int16).reshape(10, 2))
    return p


def test_wav_with_extra_chunk_is_read(tmp_path, oracle_mod):
    """A LIST chunk between fmt and data (the reference assumes a 44-byte header)."""
    data = np.arange(-500, 500, dtype=np.int16).reshape(-1, 2)
    base = tmp_path / "b.wav"
    rb.write_wav(str(base), data)
    raw = open(base, "rb").read()
    extra = b"LIST" + (6).to_bytes(4, "little") + b"INFOab"
    patched = raw[:36] + extra + raw[36:]
    patched = patched[:4] + (len(patched) - 8).to_bytes(4, "little") + patched[8:]
    p = tmp_path / "list.wav"
    p.write_bytes(patched)
    r = _run("bin_cpu", p, 5, 256, "--out", tmp_path / "o.wav", cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert np.array_equal(rb.read_wav_samples(str(tmp_path / "o.wav")), oracle_mod.mavg_i16(data.reshape(-1), 5, 2))


def test_bin_cpu_parity_stdout_and_csv(tmp_path, stereo_wav, oracle_mod):
    path, data = stereo_wav
    r = _run("bin_cpu", path, 41, 256, "--out", tmp_path / "o.wav", cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    for line in ("--- Single Thread Averager ---", "1. LATENCY BREAKDOWN (Steady State)",
                 "2. THROUGHPUT (Steady State)", "3. INITIALIZATION COST (One-time)",
                 ">> Data saved to benchmark_data.csv"):
        assert line in r.stdout
    y = rb.read_wav_samples(str(tmp_path / "o.wav"))
    assert np.array_equal(y, oracle_mod.mavg_i16(data.reshape(-1), 41, 2))
    rows = list(csv.reader(open(tmp_path / "benchmark_data.csv")))
    assert rows[0] == HEADER
    assert rows[1][:5] == ["SingleThreadCpu", "RAM", str(data.size), "41", "0"]
    assert len(rows[1]) == 14


def test_harness_wav_matches_reference_format(tmp_path):
    """generate_wav writes the canonical 44-byte PCM16 stereo header at 44.1 kHz
    (what the reference harness gets from scipy.io.wavfile.write)."""
    import scipy.io.wavfile as wav
    p = tmp_path / "h.wav"
    assert rb.generate_wav(10_000, path=str(p), seed=3)
    rate, data = wav.read(str(p))
    assert rate == 44100 and data.shape == (5000, 2) and data.dtype == np.int16
    raw = open(p, "rb").read()
    assert raw[36:40] == b"data" and int.from_bytes(raw[16:20], "little") == 16


def test_harness_sweep_tables_match_reference():
    assert [e["path"] for e in rb.EXECUTABLES] == ["./bin_cpu", "./bin_parallel", "./bin_shared", "./bin_vec2",
                                                    "./bin_vec4", "./bin_hillis", "./bin_vhillis",
                                                    "./bin_blelloch", "./bin_vblelloch"]
    assert rb.BLOCK_SIZES == [32, 64, 128, 256, 512, 1024]
    assert len(rb.GRADES) == 38 and rb.GRADES[:12] == [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 16]
    assert len(rb.INPUT_SIZES) == 100 and rb.INPUT_SIZES[0] == 5000 and rb.INPUT_SIZES[-1] == 50_000_000


@pytest.mark.parametrize("dtype,C,k", [("f32", 1, 32), ("i16", 2, 5), ("f32", 3, 1000)])
def test_bin_cpu_synthetic_matches_oracle(tmp_path, oracle_mod, dtype, C, k):
    """Synthetic north-star mode of bin_cpu (BASELINE config #1 at C=1, k=32):
    the counter-based signal regenerated on the host, filtered by the serial
    loop, equals the oracle on the oracle's own generator output."""
    n = (1 << 16) // C * C
    r = _run("bin_cpu", "-", k, 256, "--synthetic", n, "--dtype", dtype, "--channels", C, "--verify",
             "--out", tmp_path / "y.raw", cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "VERIFY: 0 mismatches" in r.stdout
    if dtype == "f32":
        x = oracle_mod.synth_f32(n)
        want = oracle_mod.mavg_f32(x, k, C)
        got = np.fromfile(tmp_path / "y.raw", dtype=np.float32)
    else:
        x = oracle_mod.synth_i16(n)
        want = oracle_mod.mavg_i16(x, k, C)
        got = np.fromfile(tmp_path / "y.raw", dtype=np.int16)
    assert np.array_equal(got, want)
    rows = list(csv.reader(open(tmp_path / "benchmark_data.csv")))
    assert rows[1][:5] == ["SingleThreadCpu", "RAM", str(n), str(k), "0"]


@pytest.mark.parametrize("args", [["--synthetic", "0"], ["--synthetic", "10", "--dtype", "f64"],
                                  ["--synthetic", "10", "--channels", "0"], ["--verify"],
                                  ["--synthetic", "2", "--channels", "3"]])
def test_synthetic_option_validation(tmp_path, args):
    r = _run("bin_vblelloch", "-", 4, 256, *args, cwd=tmp_path)
    assert r.returncode == 1, r.stdout + r.stderr


def test_harness_baseline_configs_table():
    assert {c: (b, n, g) for c, (_, b, n, g) in rb.BASELINE_CONFIGS.items()} == {
        1: ("./bin_cpu", 1 << 20, 32), 2: ("./bin_vblelloch", 1 << 26, 64), 3: ("./bin_vec4", 1 << 28, 7),
        4: ("./bin_vblelloch", 1 << 30, 4096)}
    assert rb.SHARDED_GPUS == (1, 2, 4, 8)


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", GPU_BINS)
def test_gpu_bins_bit_exact_and_csv(tmp_path, stereo_wav, oracle_mod, name):
    path, data = stereo_wav
    for grade in (1, 7, 41, 1000):
        r = _run(name, path, grade, 96, "--out", tmp_path / "o.wav", cwd=tmp_path)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "--- MEM MODE: STANDARD (Discrete) ---" in r.stdout and "--- MODE: UNIFIED (Zero-Copy) ---" in r.stdout
        y = rb.read_wav_samples(str(tmp_path / "o.wav"))
        assert np.array_equal(y, oracle_mod.mavg_i16(data.reshape(-1), grade, 2)), (name, grade)
    rows = list(csv.reader(open(tmp_path / "benchmark_data.csv")))
    assert rows[0] == HEADER
    assert [(r[0], r[1]) for r in rows[1:3]] == [(CSV_NAMES[name], "Standard"), (CSV_NAMES[name], "Unified")]
    assert all(float(r[6]) > 0 for r in rows[1:])


@pytest.mark.gpu
def test_harness_quick_sweep_verifies_every_variant(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(CLI, "run_benchmarks.py"), "--sizes", "5000", "200000",
                        "--grades", "1", "7", "64", "--blocks", "64", "256", "--verify"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "Total Failures/Crashes: 0" in r.stdout and "Output mismatches vs bin_cpu: 0" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["bin_vblelloch", "bin_blelloch"])
def test_gpu_bins_long_windows(tmp_path, oracle_mod, name):
    """One-second windows at 44.1 kHz and beyond: the 1024-thread tile and the
    look-back scan, whose workspace comes from the CLI's DspWorkspace scratch,
    in both memory modes (Standard, Unified = managed scratch too)."""
    rng = np.random.default_rng(11)
    data = rng.integers(-32768, 32767, size=(150_001, 2), dtype=np.int16)
    path = tmp_path / "long.wav"
    rb.write_wav(str(path), data)
    for grade in (5000, 44100, 70000):
        r = _run(name, path, grade, 256, "--out", tmp_path / "o.wav", cwd=tmp_path)
        assert r.returncode == 0, r.stdout + r.stderr
        y = rb.read_wav_samples(str(tmp_path / "o.wav"))
        assert np.array_equal(y, oracle_mod.mavg_i16(data.reshape(-1), grade, 2)), (name, grade)


@pytest.mark.gpu
@pytest.mark.parametrize("name,dtype,C,k", [("bin_vblelloch", "f32", 1, 64), ("bin_vec4", "f32", 1, 7),
                                            ("bin_vhillis", "f32", 2, 1000), ("bin_blelloch", "i16", 2, 44100),
                                            ("bin_parallel", "i16", 1, 9)])
def test_gpu_bins_synthetic_match_oracle(tmp_path, oracle_mod, name, dtype, C, k):
    """Synthetic mode on the device: mavg_fill_synthetic + the variant's kernel
    against the oracle (int16 bit-exact, fp32 within 1e-5 relative)."""
    n = 300_007 // C * C
    r = _run(name, "-", k, 256, "--synthetic", n, "--dtype", dtype, "--channels", C, "--verify",
             "--out", tmp_path / "y.raw", cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "4. ROOFLINE" in r.stdout and " 0 mismatches" in r.stdout
    if dtype == "f32":
        want = oracle_mod.mavg_f32(oracle_mod.synth_f32(n), k, C)
        got = np.fromfile(tmp_path / "y.raw", dtype=np.float32)
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=0)  # north_star: 1e-5 relative
    else:
        want = oracle_mod.mavg_i16(oracle_mod.synth_i16(n), k, C)
        assert np.array_equal(np.fromfile(tmp_path / "y.raw", dtype=np.int16), want)
    rows = list(csv.reader(open(tmp_path / "benchmark_data.csv")))
    assert rows[1][:3] == [CSV_NAMES[name], "Device", str(n)]


@pytest.mark.gpu
def test_harness_baseline_configs_verify():
    """The five BASELINE.json configurations through the harness: #1-#4 on the
    bin_* synthetic mode with span verification, #5 through bench.py --check on
    the GPUs present (one on the test box)."""
    r = subprocess.run([sys.executable, os.path.join(CLI, "run_benchmarks.py"), "--baseline-configs", "--verify",
                        "--max-gpus", "1"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "Failures: 0" in r.stdout
    for c in (1, 2, 3, 4, 5):
        assert f"\n#{c} " in r.stdout
    assert r.stdout.count("0 mismatches") >= 5


@pytest.mark.gpu
@pytest.mark.parametrize("name,block,want", [("bin_vblelloch", 512, 512), ("bin_vblelloch", 32, 64),
                                             ("bin_blelloch", 1024, 1024), ("bin_vhillis", 128, 128),
                                             ("bin_vec4", 1024, 1024), ("bin_shared", 64, 64),
                                             ("bin_parallel", 96, 96), ("bin_parallel", 1024, 1024)])
def test_gpu_bins_run_the_argv_block_size(tmp_path, stereo_wav, oracle_mod, name, block, want):
    """The reference launches with the argv block size (blelloch_scan_averager.cu:
    155,215-217; run_benchmarks.py:21 sweeps 32..1024): the launch each binary
    reports runs that workgroup (naive exactly, tiled kernels the next power of
    two >= one wave64), and the output is unchanged."""
    import re
    path, data = stereo_wav
    r = _run(name, path, 41, block, "--out", tmp_path / "o.wav", cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    kern = [l for l in r.stderr.splitlines() if l.startswith("Kernel: ")]  # stderr: stdout is the reference report
    assert kern and re.search(r"block=(\d+)", kern[0]).group(1) == str(want), kern
    assert np.array_equal(rb.read_wav_samples(str(tmp_path / "o.wav")), oracle_mod.mavg_i16(data.reshape(-1), 41, 2))
    rows = list(csv.reader(open(tmp_path / "benchmark_data.csv")))
    assert rows[1][4] == str(block)


# The reference's stdout, line by line: the variant's header (if it prints one:
# hillis_steele_averager.cu:205-207, profilable_parallel_averager.cu:118-121,
# profilable_sm_averager.cu:141-144), then per memory mode the mode line
# (e.g. blelloch_scan_averager.cu:237,266) and ProfileResult::print_stats
# (benchmark.h:47-68; the H2D / D2H lines only when those phases took time),
# then CsvLogger::log()'s line for the CSV row (gpu_utils.h:230).
_NUM = r"-?[0-9]+\.[0-9]{3}"
_STATS = [r"1\. LATENCY BREAKDOWN \(Steady State\)", rf"?   H2D Transfer:   {_NUM} ms",
          rf"   Kernel Compute: {_NUM} ms", rf"?   D2H Transfer:   {_NUM} ms", r"   -----------------------------",
          rf"   TOTAL LATENCY:  {_NUM} ms", r"", r"2\. THROUGHPUT \(Steady State\)",
          rf"   Kernel Bandwidth: {_NUM} GB/s", rf"   Kernel Speed:   {_NUM} Mega Samples/s",
          rf"   App BandWidth:   {_NUM} GB/s", rf"   App Speed:      {_NUM} Mega Samples/s",
          rf"   Cold Start:     {_NUM} Mega Samples/s \(Includes Init\)", r"", r"3\. INITIALIZATION COST \(One-time\)",
          rf"   Allocation:     {_NUM} ms", rf"   First Frame:    {_NUM} ms \(Cold Start\)",
          r"___________________________________", r""]
_HEADERS = {
    "bin_parallel": [r"--- SIMPLE PARALLEL AVERAGER ---", r"Samples: 12002", r"point: 41", r"block Size: 96"],
    "bin_shared": [r"--- SHARED MEMORY PARALLEL AVERAGER ---", r"Samples: 12002", r"point: 41", r"block Size: 96"],
    "bin_hillis": [r"--- Hillis Steele Averager ---", r"total samples: 12002", r"point: 41"],
}


def _report_template(name):
    lines = list(_HEADERS.get(name, []))
    for mode in (r"--- MEM MODE: STANDARD \(Discrete\) ---", r"--- MODE: UNIFIED \(Zero-Copy\) ---"):
        # CsvLogger::log() reports each row it writes (gpu_utils.h:230)
        lines += [r"", mode] + _STATS + [r">> Data saved to benchmark_data\.csv"]
    return lines


def _match_report(stdout, template):
    """Match stdout line by line; a template line starting with '?' is optional."""
    import re
    out = stdout.split("\n")
    i = 0
    for pat in template:
        optional = pat.startswith("?")
        pat = pat[1:] if optional else pat
        if i < len(out) and re.fullmatch(pat, out[i]):
            i += 1
        elif not optional:
            return f"line {i}: {out[i] if i < len(out) else '<eof>'!r} does not match {pat!r}"
    rest = [l for l in out[i:] if l != ""]
    return None if not rest else f"trailing output: {rest[:3]}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", GPU_BINS)
def test_gpu_bins_stdout_is_the_reference_report(tmp_path, stereo_wav, name):
    """stdout carries nothing but the reference's report, in its order (the
    launch description goes to stderr)."""
    path, _ = stereo_wav
    r = _run(name, path, 41, 96, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    err = _match_report(r.stdout, _report_template(name))
    assert err is None, f"{name}: {err}\n{r.stdout}"
    assert "Kernel: " in r.stderr


def test_bin_cpu_stdout_is_the_reference_report(tmp_path, stereo_wav):
    """bin_cpu's whole stdout against the reference's CPU averager report:
    header (profilable_moving_averager.cpp:51-53), one stats block (:80),
    the CSV logger's line (gpu_utils.h:230, printed by log()) -- and the
    matcher rejects extra lines."""
    path, _ = stereo_wav
    r = _run("bin_cpu", path, 41, 96, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    tmpl = [r"--- Single Thread Averager ---", r"total samples: 12002", r"point: 41"] + _STATS + [
        r">> Data saved to benchmark_data\.csv"]
    assert _match_report(r.stdout, tmpl) is None, r.stdout
    assert _match_report(r.stdout + "Kernel: x\n", tmpl) is not None
