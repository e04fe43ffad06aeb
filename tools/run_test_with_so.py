"""Runs one test function of tests/test_gpu_parity.py against an alternative library (tool):
argv[1] = the .so, argv[2] = the test name; prints PASS or FAIL (exit 0 either way)."""
import os, sys, traceback
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "divortio-lz4_amd"):
    sys.path.insert(0, os.path.join(R, p))
import lz4mi  # noqa: E402
lz4mi.LIB_PATH = os.path.abspath(sys.argv[1])
import importlib.util  # noqa: E402
spec = importlib.util.spec_from_file_location("tgp", os.path.join(R, "tests", "test_gpu_parity.py"))
m = importlib.util.module_from_spec(spec)
spec.loader.exec_module(m)
try:
    getattr(m, sys.argv[2])()
    print("PASS", sys.argv[1], sys.argv[2])
except AssertionError:
    print("FAIL", sys.argv[1], sys.argv[2], traceback.format_exc().strip().splitlines()[-1][:200])
