"""Build A/B variants of libpsrt.so with compile-time knobs (tuning only).

    python scripts/build_variants.py NAME=DEF1,DEF2 ...   -> petershirleyraytracer_amd/lib/libpsrt_NAME.so
Select one at run time with PSRT_LIB=<path>.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from petershirleyraytracer_amd import build  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition("=")
    out = os.path.join(build.LIB_DIR, f"libpsrt_{name}.so")
    build.build_lib(force=True, out=out, defines=[d for d in defs.split(",") if d])
    print(out)
