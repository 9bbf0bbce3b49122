#!/usr/bin/env python3
"""Sweep harness for the bin_* CLIs -- counterpart of the reference's
basics/run_benchmarks.py (which does not run as shipped: SyntaxError at :111).

Same sweep semantics as the reference (run_benchmarks.py:8-116):
  * EXECUTABLES: the nine ./bin_<variant> programs, bin_cpu without a block sweep
  * BLOCK_SIZES 32..1024, GRADES 1..10, 11..46 step 5, 50..1000 step 50
  * INPUT_SIZES: 100 sizes from 5,000 to 50,000,000 samples
  * per size: write a random stereo int16 WAV at 44.1 kHz, then run every
    binary x grade (skipping grade >= n) x block size, counting non-zero exit
    codes as failures; rows land in each binary's ./benchmark_data.csv
Differences: the WAV generator is seeded (reproducible), the sweep can be
restricted from the command line (--quick, --sizes, --grades, --blocks,
--bins), and --verify checks every GPU binary's filtered output against
bin_cpu's on the same WAV (all variants are bit-exact on int16).

--baseline-configs runs the five BASELINE.json configurations instead of the
WAV sweep: #1-#4 through the bin_* programs' synthetic fp32
mode (HBM-resident input, kernel-only timing, roofline line), #5 -- the
sharded signal, 2^30 samples per GPU, k=1024, (k-1)-sample RCCL halo --
through bench.py --gpus N (which starts one rank per GPU) at 1, 2, 4 and 8
GPUs, as many as the node has.

    cd digital_signal_processsing_amd/cli && python run_benchmarks.py --quick
    python run_benchmarks.py --baseline-configs --verify
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

EXECUTABLES = [
    {"name": "CPU_SingleThread", "path": "./bin_cpu", "needs_block": False},
    {"name": "Parallel_Avg", "path": "./bin_parallel", "needs_block": True},
    {"name": "SharedMem", "path": "./bin_shared", "needs_block": True},
    {"name": "Vectorized_int2", "path": "./bin_vec2", "needs_block": True},
    {"name": "Vectorized_int4", "path": "./bin_vec4", "needs_block": True},
    {"name": "HillisSteele", "path": "./bin_hillis", "needs_block": True},
    {"name": "V_HillisSteele", "path": "./bin_vhillis", "needs_block": True},
    {"name": "Blelloch", "path": "./bin_blelloch", "needs_block": True},
    {"name": "V_Blelloch", "path": "./bin_vblelloch", "needs_block": True},
]
BLOCK_SIZES = [32, 64, 128, 256, 512, 1024]
GRADES = list(range(1, 11)) + list(range(11, 51, 5)) + list(range(50, 1001, 50))
INPUT_SIZES = [int(v) for v in np.linspace(5000, 50_000_000, 100)]
TEMP_WAV = "temp_bench.wav"
REPO = os.path.dirname(os.path.dirname(HERE))

# BASELINE.json configs[0..3]: (label, binary, fp32 samples, grade)
BASELINE_CONFIGS = {
    1: ("CPU serial, N=2^20 fp32, k=32", "./bin_cpu", 1 << 20, 32),
    2: ("Blelloch scan, N=2^26 fp32, k=64, float4 loads", "./bin_vblelloch", 1 << 26, 64),
    3: ("small-window direct LDS-tiled, N=2^28 fp32, k=7", "./bin_vec4", 1 << 28, 7),
    4: ("large-window scan, N=2^30 fp32, k=4096", "./bin_vblelloch", 1 << 30, 4096),
}
# configs[4]: sharded 2^30 fp32 samples per GPU, k=1024, RCCL halo
SHARDED_GPUS = (1, 2, 4, 8)


def write_wav(path: str, data: np.ndarray, rate: int = 44100) -> None:
    """Canonical 44-byte-header PCM16 WAV (what scipy.io.wavfile writes)."""
    frames, channels = data.shape
    payload = np.ascontiguousarray(data, dtype="<i2").tobytes()
    hdr = b"RIFF" + (36 + len(payload)).to_bytes(4, "little") + b"WAVEfmt "
    hdr += (16).to_bytes(4, "little") + (1).to_bytes(2, "little") + channels.to_bytes(2, "little")
    hdr += rate.to_bytes(4, "little") + (rate * channels * 2).to_bytes(4, "little")
    hdr += (channels * 2).to_bytes(2, "little") + (16).to_bytes(2, "little")
    hdr += b"data" + len(payload).to_bytes(4, "little")
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(payload)


def read_wav_samples(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        raw = f.read()
    return np.frombuffer(raw[44:], dtype="<i2")


def generate_wav(num_samples: int, channels: int = 2, seed: int = 0, path: str = TEMP_WAV) -> bool:
    """Random stereo int16 signal of num_samples samples (num_samples/2 frames)."""
    frames = int(num_samples // channels)
    rng = np.random.default_rng(seed)
    try:
        data = rng.integers(-32768, 32767, size=(frames, channels), dtype=np.int16)
    except MemoryError:
        print(f"Could not generate {num_samples} samples.")
        return False
    write_wav(path, data)
    return True


def run_suite(sizes, grades, blocks, bins, verify=False, timeout=600) -> int:
    exes = [e for e in EXECUTABLES if bins is None or e["path"].lstrip("./") in bins]
    total = sum(len([g for g in grades if g < n]) * (len(blocks) if e["needs_block"] else 1)
                for n in sizes for e in exes)
    print("__________________________")
    print("STARTING BENCHMARK SUITE")
    print(f"Target Runs: {total}")
    print(f"Max Samples: {max(sizes)}")
    print("__________________________\n")
    start = time.time()
    counter = failures = mismatches = 0
    for n in sizes:
        print(f"\nInput Size: {n}")
        if not generate_wav(n, seed=n):
            continue
        for exe in exes:
            if not os.path.exists(exe["path"]):
                print(f"Binary not found: {exe['path']}")
                continue
            for grade in grades:
                if grade >= n:
                    continue
                for b in (blocks if exe["needs_block"] else [256]):
                    counter += 1
                    cmd = [exe["path"], TEMP_WAV, str(grade), str(b)]
                    if verify:
                        cmd += ["--out", "temp_out.wav", "--modes", "standard"]
                    try:
                        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                           universal_newlines=True, timeout=timeout)
                        if r.returncode != 0:
                            failures += 1
                            print(f"Failure: {exe['name']} (N={n}, G={grade}, B={b})")
                            print(f"Return Code: {r.returncode}")
                            print(f"Error: {r.stderr}")
                        elif verify:
                            if exe["needs_block"]:
                                ok = np.array_equal(read_wav_samples("temp_out.wav"),
                                                    read_wav_samples(f"temp_ref_{grade}.wav"))
                                if not ok:
                                    mismatches += 1
                                    print(f"MISMATCH vs bin_cpu: {exe['name']} (N={n}, G={grade}, B={b})")
                            else:
                                os.replace("temp_out.wav", f"temp_ref_{grade}.wav")
                    except Exception as e:  # noqa: BLE001 - mirror the reference's catch-all
                        failures += 1
                        print(f"Python execution failed: {e}")
                    if counter % 50 == 0:
                        print(f"{counter} runs. Elapsed: {time.time() - start:.1f}s")
        for g in grades:
            if os.path.exists(f"temp_ref_{g}.wav"):
                os.remove(f"temp_ref_{g}.wav")
    for f in (TEMP_WAV, "temp_out.wav"):
        if os.path.exists(f):
            os.remove(f)
    print("\n__________________________________")
    print("BENCHMARK COMPLETE")
    print(f"Total Runs: {counter}")
    print(f"Total Failures/Crashes: {failures}")
    if verify:
        print(f"Output mismatches vs bin_cpu: {mismatches}")
    print("Results saved to: benchmark_data.csv")
    print("__________________________________\n")
    return failures + mismatches


def _field(text: str, key: str):
    for line in text.splitlines():
        if line.strip().startswith(key):
            return line.split(":", 1)[1].strip()
    return None


def _gpu_count() -> int:
    # a child process counts the devices (torch.cuda.device_count() does not
    # initialise the GPU on this image); the harness itself stays torch-free
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, universal_newlines=True)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def run_baseline_configs(configs, verify=False, max_gpus=None, timeout=900) -> int:
    """The five BASELINE.json configurations; returns the failure count."""
    import json

    failures = 0
    rows = []
    for c in sorted(x for x in configs if x in BASELINE_CONFIGS):
        label, exe, n, grade = BASELINE_CONFIGS[c]
        cmd = [exe, "-", str(grade), "256", "--synthetic", str(n), "--dtype", "f32"]
        if verify:
            cmd.append("--verify")
        print(f"== config #{c}: {label}\n   {' '.join(cmd)}", flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True,
                           timeout=timeout)
        print(r.stdout, end="")
        if r.returncode != 0:
            failures += 1
            print(f"Failure: config #{c} rc={r.returncode}\n{r.stderr}")
            continue
        if exe == "./bin_cpu":
            ms = float(_field(r.stdout, "Kernel Compute").split()[0])
            rows.append((c, label, n / (ms * 1e-3) / 1e9, None, _field(r.stdout, "VERIFY")))
        else:
            rows.append((c, label, float(_field(r.stdout, "Gsamples/s")), float(_field(r.stdout, "of 8 TB/s peak")),
                         _field(r.stdout, "VERIFY")))
    if 5 in configs:
        have = _gpu_count() if max_gpus is None else max_gpus
        for g in [g for g in SHARDED_GPUS if g <= have]:
            bench = [os.path.join(REPO, "bench.py"), "--gpus", str(g), "--steps", "20", "--warmup", "5",
                     "--no-cpu-baseline"] + (["--check"] if verify else [])
            cmd = [sys.executable] + bench  # bench.py --gpus g starts its g ranks itself
            label = f"sharded signal, {g} x 2^30 fp32, k=1024, RCCL halo"
            print(f"== config #5 ({g} GPU): {' '.join(cmd)}", flush=True)
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True,
                               timeout=timeout, cwd=REPO)
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not lines:
                failures += 1
                print(f"Failure: config #5 at {g} GPUs rc={r.returncode}\n{r.stderr[-2000:]}")
                continue
            d = json.loads(lines[-1])
            chk = d.get("check")
            rows.append((5, label, d["value"], d["roofline"]["frac"] * 1.0,
                         None if chk is None else f"{chk['mismatches']} mismatches in {chk['slices']} slices"))
    print("\n__________________________________")
    print("BASELINE CONFIGS (Gsamples/s; fraction of 8 TB/s per GPU)")
    for c, label, gs, frac, ver in rows:
        f = "" if frac is None else f"  {frac:.3f} of HBM peak"
        v = "" if ver is None else f"  [verify: {ver}]"
        print(f"#{c} {label}: {gs:.3f} Gsamples/s{f}{v}")
    print(f"Failures: {failures}")
    print("__________________________________\n")
    return failures


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--quick", action="store_true", help="3 sizes x 5 grades x 2 block sizes")
    ap.add_argument("--sizes", type=int, nargs="*")
    ap.add_argument("--grades", type=int, nargs="*")
    ap.add_argument("--blocks", type=int, nargs="*")
    ap.add_argument("--bins", nargs="*", help="subset, e.g. bin_cpu bin_vblelloch")
    ap.add_argument("--verify", action="store_true", help="compare every GPU binary's output with bin_cpu's")
    ap.add_argument("--baseline-configs", type=int, nargs="*", metavar="N",
                    help="run BASELINE.json configs (default all: 1 2 3 4 5) instead of the WAV sweep")
    ap.add_argument("--max-gpus", type=int, default=None, help="config #5: use at most this many GPUs")
    a = ap.parse_args(argv)
    if a.baseline_configs is not None:
        os.chdir(HERE)
        return 1 if run_baseline_configs(a.baseline_configs or [1, 2, 3, 4, 5], a.verify, a.max_gpus) else 0
    sizes, grades, blocks = INPUT_SIZES, GRADES, BLOCK_SIZES
    if a.quick:
        sizes, grades, blocks = [5000, 1_000_000, 4_000_000], [1, 7, 41, 64, 1000], [64, 256]
    sizes = a.sizes or sizes
    grades = a.grades or grades
    blocks = a.blocks or blocks
    if a.verify and a.bins is not None and "bin_cpu" not in a.bins:
        a.bins = ["bin_cpu"] + a.bins
    os.chdir(HERE)
    return 1 if run_suite(sizes, grades, blocks, a.bins, a.verify) else 0


if __name__ == "__main__":
    sys.exit(main())
