"""Sanitizer runs of host code (ASan/UBSan on the CPU path).

* the C restatement (oracle/rk_ref.c) under ASan + UBSan + LeakSanitizer: every method,
  the register and wide stiff paths, ragged groups, stiff / NaN / negative walkers, MH
  with Philox and replay draws (tests/sanitize/rkref_driver.c);
* the same driver under MemorySanitizer (clang, origins tracked): no uninitialised read in
  the restated algorithms — the lockstep BDF group and the MH kernels' per-lane BDF at
  S = 4 and 8 included — so a device result that depends on code shape is not an
  algorithm reading undefined state (profiles/NOTES.md, round 5);
* the C-ABI's host code (capi/rtc/comm built with host-side ASan + UBSan, device code as
  shipped): validation and error paths and a hipRTC compile on the CPU; the full device
  path (every method, MH in every RNG mode, resume, a run-time compiled model with its
  lazily built stiff kernels) on the GPU.
Executables are built by __graft_entry__.build() (make -C tests/sanitize)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")
# the box preloads a library of its own ahead of libasan: keep ASan's link-order check off
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _exe(name):
    path = os.path.join(SAN, "build", name)
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", SAN, f"build/{name}"], check=True)
    return path


def test_rk_ref_under_asan_ubsan_lsan():
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", OMP_NUM_THREADS="2")
    r = subprocess.run([_exe("rkref_asan")], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "SANITIZE OK" in r.stdout, r.stderr[-4000:]


def test_rk_ref_under_msan():
    r = subprocess.run([_exe("rkref_msan")], env=dict(os.environ, MSAN_OPTIONS="halt_on_error=1"),
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0 and "SANITIZE OK" in r.stdout, r.stderr[-4000:]


def test_c_abi_host_code_under_asan_ubsan_error_paths():
    r = subprocess.run([_exe("capi_asan")], env=ENV, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "SANITIZE OK" in r.stdout, r.stderr[-4000:]


@pytest.mark.gpu
def test_c_abi_host_code_under_asan_ubsan_on_device():
    r = subprocess.run([_exe("capi_asan"), "device"], env=ENV, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "SANITIZE OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
