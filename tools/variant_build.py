"""Build an A/B copy of libaidfp.so in which ONE source file gets extra compiler flags.

usage: python tools/variant_build.py NAME FILE FLAG...   -> audio-ident_amd/build/NAME/libaidfp.so
(the other objects are the product build's audio-ident_amd/build/*.o; run build_ext.py first)
"""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "audio-ident_amd"))
import build_ext as B  # noqa: E402

name, src, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
B.build()
out = B.OBJ / name
out.mkdir(parents=True, exist_ok=True)
obj = out / (src + ".o")
cmd = [B.HIPCC, *B.FLAGS, *B.FILE_FLAGS.get(src, []), *extra, "-c", str(B.CSRC / src), "-o", str(obj)]
if src.endswith(".cpp"):
    cmd = [B.HIPCC, *B.FLAGS, *extra, "-x", "hip", "-c", str(B.CSRC / src), "-o", str(obj)]
subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
objs = [obj if s == src else B.OBJ / (s + ".o") for s in B.SOURCES]
lib = out / "libaidfp.so"
subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs),
                "-L/opt/rocm/lib", "-lrccl"], check=True)
print(lib)
