"""Build the instrumented library variants used by tools/gpu_quick.sh and
tools/llt_items.py (variants/*.so, git-ignored, shipped to the GPU box):
lib_T.so  -DM3S_LLT_TIMING=1 (phase stamps), lib_I.so -DM3S_LLT_ITEMS=1 (per-item stamps)."""
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

os.makedirs(os.path.join(ROOT, "variants"), exist_ok=True)
for name, flag in (("lib_T.so", "-DM3S_LLT_TIMING=1"), ("lib_I.so", "-DM3S_LLT_ITEMS=1")):
    subprocess.check_call([g._hipcc(), "--offload-arch=gfx950", "-O3", "-fno-slp-vectorize", "-std=c++17", "-fPIC",
                           "-shared", flag, "-I", os.path.join(ROOT, "include"), *g.SOURCES, "-o",
                           os.path.join(ROOT, "variants", name)])
