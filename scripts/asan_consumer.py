"""Host-side sanitizer pass over the drop-in path's host code (this container
only; no GPU): every mOS consumer scenario of tests/test_mos_consumer.py, in the
8- and 16-byte record forms, through oracle/_ref/asan/mos_app_emul -- mOS itself
over gpu_module_func with the CPU stand-in for the GPU, the backend
(gpu_module.c) and the consumer (mos_rx.c) built with AddressSanitizer and
UBSan (make -C oracle asan).  Each scenario must give the same results as in
the suite and the sanitizers must report nothing.

Usage: python3 scripts/asan_consumer.py [scenario ...]   (log: stdout)"""
import os
import pathlib
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_mos_consumer as T  # noqa: E402

EXE = os.path.join(ROOT, "oracle", "_ref", "asan", "mos_app_emul")
# leaks: mOS frees little at exit (its pools live for the process); the harness
# preloads a library of its own, so ASan's link-order check is relaxed
os.environ["ASAN_OPTIONS"] = "detect_leaks=0:verify_asan_link_order=0:abort_on_error=0:halt_on_error=1"
os.environ["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"


def main():
    names = sys.argv[1:] or sorted(T.SCENARIOS)
    bad = 0
    for name in names:
        for form in ("c8", "rec16"):
            with tempfile.TemporaryDirectory() as d:
                try:
                    pp, gpu = T.compare_modes(EXE, pathlib.Path(d), name, form)
                    T._check_scenario(name, pp, gpu, form)
                    print(f"ok   {name} [{form}]", flush=True)
                except AssertionError as e:
                    bad += 1
                    print(f"FAIL {name} [{form}]: {str(e)[-3000:]}", flush=True)
    print(f"{bad} failing of {2 * len(names)}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
