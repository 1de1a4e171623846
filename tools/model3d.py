"""Scale model of the 3D grid factorization (pdgstrf3d) from measured
per-layer phase times on ONE GPU.

For each depth Pz, every layer's plan (1x1 layers, the coarse reference
partition the grid benches use) is built and factored alone on the GPU with
SLU_3D_SOLO=1 (its ancestor reductions pack / add but exchange nothing), and
its per-phase device times are read from the plan stats.  The predicted
factorization time on Pz GPUs is the critical path

    T(Pz) = sum_p [ max over the layers active in phase p of t_phase(z, p) ]
          + sum_p [ max over the pairs of phase p of bytes_p / B_xgmi ]

(phase p = forest level p, 0 = leaves; a layer z is active in phase p when
z % 2^p == 0; the pack / add kernels are inside the measured phase times).
The measured 1-GPU time of the same partition (Pz = 1) is the reference
point.  Prints one JSON object.

    python tools/model3d.py [--nx 100] [--pz 2,4,8] [--bw 50,100]
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def log(m):
    print(f"[model3d {time.strftime('%H:%M:%S')}] {m}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=100)
    ap.add_argument("--pz", default="2,4,8")
    ap.add_argument("--bw", default="50,100", help="xGMI point-to-point GB/s to model")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    os.environ["SLU_3D_SOLO"] = "1"
    import bench
    from superlu_dist_amd.engine import Comm, Plan

    t0 = time.time()
    A, S, lu, perm = bench.build_lu("lap3d", args.nx, 1, 1, 0, 0, "grid", "reference", coarse=True)
    anorm = bench.one_norm(A)
    log(f"front-end {time.time() - t0:.1f} s, {S.nsupers} supernodes (coarse)")

    def never(ops):
        raise RuntimeError("SLU_3D_SOLO plans exchange nothing")

    def run(comm):
        p = Plan(lu, comm=comm, timing=1)
        p.upload()
        p.snapshot()
        best = None
        for _ in range(args.reps):
            p.restore()
            p.sync()
            t = time.perf_counter()
            p.factor(anorm)
            p.sync()
            dt = (time.perf_counter() - t) * 1e3
            st = p.stats()
            if best is None or dt < best[0]:
                best = (dt, st)
        del p
        gc.collect()
        return best

    base_ms, st1 = run(None)
    log(f"Pz=1: {base_ms:.1f} ms")
    out = {"nx": args.nx, "nsupers": int(S.nsupers), "t1_ms": round(base_ms, 2),
           "flops": float(st1["schur_flops"] + st1["panel_flops"]), "models": []}
    for pz in (int(x) for x in args.pz.split(",")):
        maxlvl = pz.bit_length()
        layers = []
        for z in range(pz):
            comm = Comm.host_p2p3d(1, 1, pz, z, 0, never)
            ms, st = run(comm)
            last = int(st["phase_last"])
            layers.append({"z": z, "wall_ms": round(ms, 2), "phase_last": last,
                           "phase_ms": [round(x, 3) for x in st["t_phase_ms"][:last + 1]],
                           "zred_gb": [round(x / 1e9, 4) for x in st["zred_bytes"][:maxlvl - 1]],
                           "factored": int(st["nsupers"]),
                           "flops": float(st["schur_flops"] + st["panel_flops"])})
            log(f"Pz={pz} layer {z}: {ms:.1f} ms, phases {layers[-1]['phase_ms']}")
            del comm
        comp = []
        red_gb = []
        for p in range(maxlvl):
            act = [L for L in layers if L["z"] % (1 << p) == 0]
            comp.append(max(L["phase_ms"][p] for L in act))
            if p < maxlvl - 1:
                red_gb.append(max(L["zred_gb"][p] for L in act))
        for bw in (float(b) for b in args.bw.split(",")):
            t = sum(comp) + sum(g / bw * 1e3 for g in red_gb)
            out["models"].append({"pz": pz, "bw_gbs": bw, "t_ms": round(t, 2),
                                  "speedup": round(base_ms / t, 2),
                                  "compute_ms_per_phase": [round(c, 2) for c in comp],
                                  "reduce_gb_per_phase": red_gb})
        out.setdefault("layers", {})[pz] = layers
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
