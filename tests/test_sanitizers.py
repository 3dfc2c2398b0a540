"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

build/host_sanitize (Makefile; tools/host_sanitize.cpp) links the host-side
sources of libbert.so that parse untrusted input — the GGUF reader
(gguf_io.cpp, reference gguf.h / bert.cpp:173-204 replaced), the WordPiece
tokenizer (tokenizer.cpp) — and the GGUF writer + Q4 quantiser
(quantize*.cpp, bert_model_quantize) with -fsanitize=address,undefined
-fno-sanitize-recover=all: any finding aborts the process, so a clean exit
status is the assertion.  The GGUF reader is fed truncated and corrupted
copies of a valid model (counts, sizes, offsets, types, dimensions), the
tokenizer random byte strings.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "build", "host_sanitize")


@pytest.fixture(scope="module")
def san(tmp_path_factory):
    subprocess.run(["make", "-s", "-C", REPO, "build/host_sanitize"], check=True)
    d = tmp_path_factory.mktemp("san")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    def run(*args):
        r = subprocess.run([EXE, *map(str, args)], capture_output=True, text=True, env=env, timeout=300)
        assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
        return r
    return d, run


def test_synth_parse_tokenize_quantize(san):
    d, run = san
    f16, q40, q41 = d / "m.gguf", d / "m_q4_0.gguf", d / "m_q4_1.gguf"
    assert run("synth", f16).returncode == 0
    assert run("parse", f16).returncode == 0
    r = run("tok", f16, "Hello, world!", "Québec 北京", "x" * 300, "")
    assert r.returncode == 0 and r.stdout.count(":") == 4
    assert run("quant", f16, q40, 2).returncode == 0 and run("parse", q40).returncode == 0
    assert run("quant", f16, q41, 3).returncode == 0 and run("parse", q41).returncode == 0


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gguf_reader_corrupted_inputs(san, seed):
    d, run = san
    f = d / f"fz{seed}.gguf"
    assert run("synth", f).returncode == 0
    q = d / f"fz{seed}_q4.gguf"
    assert run("quant", f, q, 2 if seed % 2 else 3).returncode == 0
    for src in (f, q):
        r = run("fuzz", src, seed, 1500)
        assert r.returncode == 0 and "fuzz: 1500 variants" in r.stdout, r.stdout + r.stderr[-2000:]


def test_tokenizer_random_bytes(san):
    d, run = san
    f = d / "tk.gguf"
    assert run("synth", f).returncode == 0
    r = run("tokfuzz", f, 9, 3000)
    assert r.returncode == 0 and "tokfuzz:" in r.stdout
