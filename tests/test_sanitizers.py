"""Host-code sanitizers (GPU ASan is not available on this pool): the oracle
restatement and the CLI's WAV parser built with -fsanitize=address,undefined
and driven over edge shapes and malformed / truncated WAV files."""
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g", "-O1"]

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")


def _env():
    e = dict(os.environ)
    e["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    e["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    e.pop("LD_PRELOAD", None)
    return e


def test_oracle_edges_asan_ubsan(tmp_path):
    exe = tmp_path / "oracle_edges"
    subprocess.run(["gcc", *SAN, "-fopenmp", "-std=c11", "-o", str(exe), os.path.join(HERE, "sanitize", "oracle_edges.c"),
                    os.path.join(ROOT, "oracle", "mavg_oracle.c")], check=True)
    r = subprocess.run([str(exe)], env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True)
    assert r.returncode == 0 and "edges ok" in r.stdout, r.stderr[-3000:]


def _wav(frames, channels=2, bits=16, fmt_size=16, extra=b"", truncate=None):
    payload = np.arange(frames * channels, dtype="<i2").tobytes()
    fmt = (1).to_bytes(2, "little") + channels.to_bytes(2, "little") + (44100).to_bytes(4, "little")
    fmt += (44100 * channels * 2).to_bytes(4, "little") + (channels * 2).to_bytes(2, "little")
    fmt += bits.to_bytes(2, "little") + b"\0" * (fmt_size - 16)
    body = b"WAVE" + b"fmt " + fmt_size.to_bytes(4, "little") + fmt + extra + b"data"
    body += len(payload).to_bytes(4, "little") + payload
    raw = b"RIFF" + len(body).to_bytes(4, "little") + body
    return raw if truncate is None else raw[:truncate]


def test_wav_parser_asan_ubsan_on_malformed_files(tmp_path):
    exe = tmp_path / "wav_fuzz"
    subprocess.run(["g++", *SAN, "-std=c++17", "-o", str(exe), os.path.join(HERE, "sanitize", "wav_fuzz.cpp")],
                   check=True)
    good = _wav(100)
    cases = {
        "good.wav": good,
        "list.wav": _wav(10, extra=b"LIST" + (5).to_bytes(4, "little") + b"abcde\0"),
        "fmt18.wav": _wav(10, fmt_size=18),
        "u8.wav": _wav(10, bits=8),
        "empty.wav": b"",
        "riff_only.wav": b"RIFF\0\0\0\0WAVE",
        "huge_fmt.wav": b"RIFF\0\0\0\0WAVEfmt \xff\xff\xff\x7f",
        "short_fmt.wav": b"RIFF\0\0\0\0WAVEfmt \x04\0\0\0abcd",
        "huge_data.wav": good[:40] + b"\xff\xff\xff\xff" + good[44:],
        "odd_chunk.wav": _wav(4, extra=b"junk" + (3).to_bytes(4, "little") + b"xyz\0"),
    }
    for cut in (11, 20, 30, 43, 45, 101):
        cases[f"trunc{cut}.wav"] = good[:cut]
    rng = np.random.default_rng(0)
    for i in range(40):  # random byte flips in the header
        b = bytearray(good)
        for _ in range(3):
            b[int(rng.integers(0, 44))] = int(rng.integers(0, 256))
        cases[f"flip{i}.wav"] = bytes(b)
    paths = []
    for name, data in cases.items():
        p = tmp_path / name
        p.write_bytes(data)
        paths.append(str(p))
    r = subprocess.run([str(exe), *paths], env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       universal_newlines=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    ok = int(r.stdout.split("ok=")[1].split()[0])
    assert ok >= 3  # good, list, fmt18 (and odd_chunk) parse
