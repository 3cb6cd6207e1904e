"""The C++ facade (include/ebpf_discovery_amd.hpp) compiled as INTEGRATION.md's call sites
would be: a real g++ build against the C header and libebd_amd.so, so a header or struct
mismatch between the ABI and a C++ caller fails here (not only through ctypes).

CPU: batch packing and the error path (no GPU: construction throws ebdamd::Error).
GPU: the Discovery poll loop over an in-memory EventSource (config 1, kernel session delete,
report + clear, network counters with an overridden clock); see tests/cpp/facade_test.cpp."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "facade_test")


def _binary():
    # built by __graft_entry__.build(); make is a no-op when it is up to date
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True, capture_output=True, timeout=300)
    return BIN


def test_cpp_facade_cpu_error_path():
    out = subprocess.run([_binary(), "cpu"], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, HIP_VISIBLE_DEVICES="-1"))
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr[-2000:]


@pytest.mark.gpu
def test_cpp_facade_discovery_loop_on_gpu():
    out = subprocess.run([_binary(), "gpu"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr[-2000:]
