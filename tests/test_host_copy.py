"""The coalescer's staging copy (csrc/rs_host_copy.cpp, streaming stores): bytes and
bounds against memcpy for every length class and alignment (CPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stage_copy_matches_memcpy_and_stays_in_bounds(tmp_path):
    exe = str(tmp_path / "test_host_copy")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "test_host_copy.cpp"),
                    os.path.join(ROOT, "replication_erasurecoding_object_store_amd", "csrc", "rs_host_copy.cpp"),
                    "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)  # both copy modes
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
