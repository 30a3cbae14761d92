"""Diagnostic: hand-off latency and producer skew of the packed BiRNN kernels (fwd; `bwd`: BPTT).

Builds a separate library with -DRNN_TRACE (never the shipped one); every workgroup
records s_memrealtime (100 MHz) at its publish and at its completed poll, per step.
Prints, over steps and groups: publish skew across the NG producers of a group, and
latency from the LAST producer's publish (step s-1) to each consumer's poll completion."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dl4ss_amd import build as B  # noqa: E402

TAG = os.environ.get("RNN_TAG", "")
LIB = os.path.join(ROOT, "dl4ss_amd", f"libdl4ss_hip_trace{TAG}.so")


def build():
    od = f"/tmp/trace_obj{TAG}"
    os.makedirs(od, exist_ok=True)
    objs = []
    for f in sorted(os.listdir(B.CSRC)):
        if f.endswith(".hip"):
            o = f"{od}/{f[:-4]}.o"
            subprocess.run([B.HIPCC, *B.FLAGS, *B.FILE_FLAGS.get(f, []), "-DRNN_TRACE", *sys.argv[2:], "-I", B.CSRC,
                            "-c", os.path.join(B.CSRC, f), "-o", o], check=True)
            objs.append(o)
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", LIB, *B.LINK], check=True)


def main():
    os.environ["DL4SS_LIB"] = LIB
    import torch
    from dl4ss_amd import _lib, engine

    dev = torch.device("cuda")
    Bsz, T, H = 32, 251, 300
    net = engine.SepNet(cell="lstm", num_layers=1, device=dev)
    tr = engine.SepTrainer(net, Bsz, 2, 32000, precision="bf16")
    grid = 240
    buf = torch.zeros(grid * T * 4, dtype=torch.int64, device=dev)
    lib = _lib.lib()
    lib.dl4ss_debug_set_stamps.argtypes = [ctypes.c_void_p]
    lib.dl4ss_debug_set_stamps(ctypes.c_void_p(buf.data_ptr()))
    x = torch.randn(Bsz, T, 129, device=dev)
    tr.spk.zero_()  # valid speaker ids for the query gather
    bwd = "bwd" in sys.argv
    for _ in range(3):
        buf.zero_()
        tr.forward(feats=x)
        torch.cuda.synchronize()
    if bwd:  # BPTT of the same layer (slot 3 = cell phase start after the first barrier)
        tr.dq.normal_()
        tr.dPreb.normal_()
        for _ in range(2):
            buf.zero_()
            tr.backward()
            torch.cuda.synchronize()
    tb = buf.view(grid, T, 4).cpu().double() * 10.0  # ns
    NG = 15
    ngroups = grid // NG
    # group_of(): ngroups % 8 == 0 -> x = bid & 7, y = bid >> 3, group = x * (ngroups/8) + y / NG, w = y % NG
    members = [[] for _ in range(ngroups)]
    for bid in range(grid):
        xx, yy = bid & 7, bid >> 3
        members[xx * (ngroups // 8) + yy // NG].append(bid)
    lat, skew, step, rtt, start_to_last, nospin = [], [], [], [], [], 0
    for g in range(ngroups):
        m = members[g]
        pub = tb[m, :, 0]
        seen = tb[m, :, 1]
        for s in range(2, T - 1):
            last = pub[:, s - 1].max()
            skew.append(float(pub[:, s - 1].max() - pub[:, s - 1].min()))
            lat.extend((seen[:, s] - last).tolist())
            step.append(float(pub[:, s].max() - pub[:, s - 1].max()))
            st0, first = tb[m, s, 2], tb[m, s, 3]
            for i in range(len(m) if not bwd else 0):
                if first[i] > 0:
                    rtt.append(float(first[i] - st0[i]))
                else:
                    nospin += 1
                start_to_last.append(float(last - st0[i]))
    import statistics as st
    q = lambda v, p: sorted(v)[int(p * (len(v) - 1))]
    print(f"step period (max publish to max publish) ns: median {st.median(step):.0f}  p10 {q(step, .1):.0f}  p90 {q(step, .9):.0f}")
    print(f"publish skew across producers ns: median {st.median(skew):.0f}  p90 {q(skew, .9):.0f}")
    if bwd:  # slots: 0 publish issued (wave 3), 1 poll complete (wave 4), 2 poll start, 3 cell start (after B1)
        print(f"last publish -> poll complete (wave 4) ns: median {st.median(lat):.0f}  p10 {q(lat, .1):.0f}  "
              f"p90 {q(lat, .9):.0f}  min {min(lat):.0f}")
        b1 = []
        for g in range(ngroups):
            m = members[g]
            for s in range(2, T - 1):
                last = tb[m, s - 1, 0].max()
                b1.extend((tb[m, s, 3] - last).tolist())
        print(f"last publish -> cell start (B1 exit) ns: median {st.median(b1):.0f}  p90 {q(b1, .9):.0f}")
        cp = [float(tb[m, s, 0] - tb[m, s, 3]) for m in range(grid) for s in range(2, T - 1)]
        print(f"cell start -> own publish issued ns: median {st.median(cp):.0f}  p90 {q(cp, .9):.0f}")
        return
    print(f"first sweep round trip (poll start -> first re-poll) ns: median {st.median(rtt):.0f} p90 {q(rtt, .9):.0f}; "
          f"polls satisfied by the first sweep: {nospin}")
    print(f"poll start -> last producer publish ns: median {st.median(start_to_last):.0f}")
    print(f"last publish -> poll complete ns: median {st.median(lat):.0f}  p10 {q(lat, .1):.0f}  p90 {q(lat, .9):.0f}  min {min(lat):.0f}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        main()
