"""The ring planner (pure C, csrc/pg_plan.c) built with AddressSanitizer and
UndefinedBehaviorSanitizer and driven over a grid of shapes (tests/c/plan_fuzz.c):
no invalid access, no UB, every step's offsets inside its buffer.  Host code
only -- GPU sanitizers are not available on the MI355X pool."""
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_planner_clean_under_asan_ubsan(tmp_path):
    exe = tmp_path / "plan_fuzz"
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "c" / "plan_fuzz.c"),
                    str(ROOT / "rdma-ring-collectives_amd" / "csrc" / "pg_plan.c"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.returncode, r.stdout[-500:], r.stderr[-2000:])
