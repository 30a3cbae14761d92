"""Diagnostic: per-phase cycle shares of the persistent BiRNN kernels.

Builds a separate library with -DRNN_STAMPS (never the shipped one), runs one
BiLSTM layer fwd + bwd at the bench shape and prints, per role thread, the
average cycles per timestep spent in each phase."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dl4ss_amd import build as B  # noqa: E402

# extra -D flags for experiment variants: RNN_DEFS="-DFOO -DBAR", library suffixed by RNN_TAG
DEFS = os.environ.get("RNN_DEFS", "").split()
LIB = os.path.join(ROOT, "dl4ss_amd", f"libdl4ss_hip_stamps{os.environ.get('RNN_TAG', '')}.so")


def build_stamps():
    objs = []
    od = f"/tmp/stamps_obj{os.environ.get('RNN_TAG', '')}"
    os.makedirs(od, exist_ok=True)
    for f in sorted(os.listdir(B.CSRC)):
        if f.endswith(".hip"):
            o = f"{od}/{f[:-4]}.o"
            subprocess.run([B.HIPCC, *B.FLAGS, "-DRNN_STAMPS", *DEFS, "-I", B.CSRC, "-c", os.path.join(B.CSRC, f), "-o", o],
                           check=True)
            objs.append(o)
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", LIB, *B.LINK], check=True)


def main():
    if not os.path.exists(LIB) or "--rebuild" in sys.argv:
        build_stamps()
    os.environ["DL4SS_LIB"] = LIB
    import ctypes
    import torch
    from dl4ss_amd import _lib, engine

    dev = torch.device("cuda")
    Bsz, T, H = 32, 251, 300
    # two layers: the forward stamps are the last forward launch's (layer 1, the 600-wide fused
    # projection, as 3 of the 4 C2 layers), the BPTT stamps the last BPTT launch's (layer 0)
    net = engine.SepNet(cell="lstm", num_layers=int(os.environ.get("STAMP_LAYERS", "2")), device=dev)
    prec = "bf16" if "--bf16" in sys.argv else "fp32"
    tr = engine.SepTrainer(net, Bsz, 2, 32000, precision=prec)
    stamps = torch.zeros(240 * 16, dtype=torch.int64, device=dev)
    lib = _lib.lib()
    lib.dl4ss_debug_set_stamps.argtypes = [ctypes.c_void_p]
    lib.dl4ss_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
    x = torch.randn(Bsz, T, 129, device=dev)
    tr.spk.zero_()  # valid speaker ids for the query gather
    if getattr(tr, "fast", False):
        tr.dPreb.normal_()
    for rep in range(2):
        stamps.zero_()
        tr.forward(feats=x)
        torch.cuda.synchronize()
        fw = stamps.view(240, 16).double().cpu() / T
        stamps.zero_()
        tr.dq.normal_()
        (tr.Vb if getattr(tr, 'fast', False) else tr.V).normal_()
        tr.backward()
        torch.cuda.synchronize()
        bw = stamps.view(240, 16).double().cpu() / T
    # slot i = cycles from the previous stamp to STAMP(i) (birnn.hip): forward cell waves
    # B2 -> gates (5) -> publish store issued (6) -> saved-state stores (4); BPTT cell waves
    # B2 -> MFMA + transpose (4) -> granule publish (5) -> dG stores (6); BPTT cell phase B1 ->
    # operand / partial-sum reads (7) -> math and the bf16 dgh image (2)
    names_f = ["gather", "bar1", "matvec", "bar2", "saves", "gates", "publish"]
    names_b = ["gather", "bar1", "cell_math", "bar2", "matvec/mfma", "publish", "dg_stores", "cell_reads"]
    print(f"precision {prec}")
    for title, st, names in (("fwd", fw, names_f), ("bwd", bw, names_b)):
        for role, off in (("thread0 (cell/publish)", 0), ("thread256 (gather)", 8)):
            m = st[:, off:off + len(names)].mean(0)
            tot = float(m.sum())
            print(f"{title} {role}: total {tot:.0f} cyc/step = " +
                  ", ".join(f"{n} {float(v):.0f}" for n, v in zip(names, m)))


if __name__ == "__main__":
    main()
