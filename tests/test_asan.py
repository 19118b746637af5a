"""CPU: the host-only C++ of libcapgen (tune-table parser, parameter-arena layout + reference-name
table, SCST n-gram scorer, run-time switch registry) built with -fsanitize=address,undefined and
driven with valid, adversarial and random inputs (tests/asan_host.cpp, make asan)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "image-caption_amd", "csrc")


def test_host_cpp_clean_under_asan_ubsan():
    subprocess.run(["make", "-C", CSRC, "asan"], check=True, capture_output=True, timeout=600)
    exe = os.path.join(REPO, "image-caption_amd", "capgen", "asan_host")
    env = {k: v for k, v in os.environ.items() if not k.startswith("CAPGEN_")}
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    out = subprocess.run([exe, os.path.join(REPO, "image-caption_amd", "capgen", "tune_gfx950.txt")],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "asan_host: ok" in out.stdout
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr
