"""Experiment helper: build a variant of libdl4ss_hip.so with extra -D flags.

  python tools/variant_lib.py TAG -DFOO -DBAR   ->  dl4ss_amd/libdl4ss_hip_TAG.so
Use it with DL4SS_LIB=dl4ss_amd/libdl4ss_hip_TAG.so (never the shipped library)."""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dl4ss_amd import build as B  # noqa: E402


def main(tag, defs):
    """--minimal: recompile only birnn.hip, with -DRNN_EXP_MINIMAL (the packed BC = 4 kernels of the
    C2 / C4 step at B = 32 only), and link it with the shipped build's other objects (python -m
    dl4ss_amd.build first): a recurrence variant in well under a minute."""
    od = f"/tmp/variant_obj_{tag}"
    os.makedirs(od, exist_ok=True)
    srcs = sorted(f for f in os.listdir(B.CSRC) if f.endswith(".hip"))
    minimal = "--minimal" in defs
    if minimal:
        defs = [d for d in defs if d != "--minimal"] + ["-DRNN_EXP_MINIMAL"]
    # --only=a.hip,b.hip: recompile just those sources, link the shipped build's other objects
    only = [d.split("=", 1)[1].split(",") for d in defs if d.startswith("--only=")]
    only = only[0] if only else (["birnn.hip"] if minimal else None)
    defs = [d for d in defs if not d.startswith("--only=")] + ["-DDL4SS_VARIANT_BUILD"]

    def comp(f):
        if only is not None and f not in only:
            return os.path.join(B.OBJ, f[:-4] + ".o")
        o = f"{od}/{f[:-4]}.o"
        subprocess.run([B.HIPCC, *B.FLAGS, *B.FILE_FLAGS.get(f, []), *defs, "-I", B.CSRC, "-c",
                        os.path.join(B.CSRC, f), "-o", o], check=True)
        return o

    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, srcs))
    lib = os.path.join(ROOT, "dl4ss_amd", f"libdl4ss_hip_{tag}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", lib, *B.LINK], check=True)
    print(lib)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
