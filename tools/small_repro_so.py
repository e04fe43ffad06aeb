"""tools/small_repro.py with an alternative library (tool): argv[1] = the .so, argv[2] = the dump."""
import os, runpy, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "divortio-lz4_amd"))
import lz4mi  # noqa: E402
lz4mi.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = [sys.argv[0], sys.argv[2]]
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "small_repro.py"), run_name="__main__")
