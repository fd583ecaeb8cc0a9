"""VALU issue analysis of the sweep kernel from rocprofv3 counter passes.

    python tools/valu_busy.py <valuclass dir> <valubusy dir> [kernel substring] [--mix valu_mix.txt]

valuclass pass: SQ_INSTS_VALU + the class counters SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, INT32, INT64,
SQ_WAVES; valubusy pass: SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE, SQ_WAVES
(tools/gpu_session.sh steps valuclass / valubusy).  Per wave of the kernel it prints the instruction
mix by class, the VALU-active cycles per VALU instruction (SQ_ACTIVE_INST_VALU counts quad-cycles,
MI355X_MICROARCH.md), the wave lifetime, and the fraction of SIMD time the VALU is issuing:
  busy = sum over waves of VALU-active cycles / (1024 SIMDs x kernel cycles),
kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs).  With --mix it sets the
measured VALU-active cycles per instruction beside the microbenchmark's per-SIMD issue costs
(tools/ubench/valu_mix.hip) at the kernel's waves per SIMD.
"""
import collections
import csv
import glob
import os
import sys


def load(d, sub):
    agg = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter*.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if sub in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    mix = sys.argv[sys.argv.index("--mix") + 1] if "--mix" in sys.argv else None
    if mix in args:
        args.remove(mix)
    cls_dir, busy_dir = args[0], args[1]
    sub = args[2] if len(args) > 2 else "bf_pairb"
    c, b = load(cls_dir, sub), load(busy_dir, sub)
    waves = c["SQ_WAVES"]
    valu = c["SQ_INSTS_VALU"] / waves
    print(f"kernel ~ {sub!r}: {waves:.0f} waves per launch, {valu:.0f} VALU instructions per wave")
    classes = ["FMA_F64", "MUL_F64", "ADD_F64", "TRANS_F64", "INT32", "INT64"]
    known = 0.0
    for k in classes:
        v = c.get("SQ_INSTS_VALU_" + k, 0.0) / waves
        known += v
        print(f"  {k:10s} {v:8.0f}  ({v / valu:5.1%})")
    cvt = b.get("SQ_INSTS_VALU_CVT", 0.0) / b["SQ_WAVES"]
    print(f"  {'CVT':10s} {cvt:8.0f}")
    print(f"  {'other':10s} {valu - known - cvt:8.0f}  (moves, DPP moves, selects, min/max, ...)")
    act = b["SQ_ACTIVE_INST_VALU"] * 4 / b["SQ_WAVES"]  # cycles per wave
    life = b["SQ_WAVE_CYCLES"] * 4 / b["SQ_WAVES"]
    kcyc = b["GRBM_GUI_ACTIVE"] / 8
    busy = b["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * kcyc)
    print(f"VALU-active cycles per wave {act:.0f} = {act / valu:.2f} per VALU instruction; wave lifetime {life:.0f} "
          f"cycles (VALU-active share {act / life:.2f})")
    print(f"kernel {kcyc:.0f} cycles (GRBM_GUI_ACTIVE / 8); SIMD VALU busy = {busy:.3f}")
    if mix:
        print("microbenchmark issue cost per wave-instruction per SIMD (tools/ubench/valu_mix):")
        for line in open(mix):
            if line.strip() and not line.startswith("cycles"):
                print("  " + line.rstrip())


if __name__ == "__main__":
    main()
