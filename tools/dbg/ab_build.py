import sys
sys.path.insert(0, "/root/repo")
from cilium_amd import build
for name, defs in (("nopol", ["AB_NOPOL"]), ("noctw", ["AB_NOCTW"]), ("noct", ["AB_NOCT"]), ("base", [])):
    build.build(force=True, out=f"/root/repo/_ab/{name}/libcilium_hip.so", defines=defs)
