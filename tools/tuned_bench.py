"""bench.py with the legacy GPAD_* tuning knobs of the environment applied to its handles
(tools/tune_env.py -> gpad_set_option).  For A/B runs only (tools/ab.sh); bench.py itself, like
the library, reads no tuning environment."""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import tune_env  # noqa: E402,F401

sys.argv[0] = os.path.join(HERE, "..", "bench.py")
runpy.run_path(sys.argv[0], run_name="__main__")
