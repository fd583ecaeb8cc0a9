"""Static instruction mix of gfx950 kernels in a hipcc --save-temps .s file.

    python tools/isa_stats.py FILE.s [substring-of-kernel-name ...]

For each kernel whose mangled or demangled name contains every substring: VGPR /
AGPR / SGPR counts, scratch bytes, occupancy (waves per SIMD) and the count of
instructions by class (fp64 VALU, other VALU, DPP, LDS, global, scalar, branches).
Static counts: a fully unrolled straight-line kernel executes each instruction once
per wave, so these are the per-wave VALU budgets the DESIGN.md roofline uses.
"""
import collections
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return out.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def classify(op):
    if op.startswith("v_"):
        if "_dpp" in op or op.endswith("dpp"):
            return "dpp"
        if op.startswith(("v_mfma", "v_smfmac")):
            return "mfma"
        if "_f64" in op or op in ("v_rsq_f64", "v_ldexp_f64"):
            return "valu_f64"
        if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            return "lane_xfer"
        if op.startswith(("v_mov_b32", "v_mov_b64", "v_cndmask")):
            return "valu_mov"
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path = sys.argv[1]
    subs = sys.argv[2:]
    lines = open(path).read().splitlines()
    # kernel bodies: from "<name>:" (after .type @function) to .Lfunc_end
    kernels = {}
    cur = None
    for ln in lines:
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
        if m:
            cur = m.group(1)
            kernels[cur] = {"body": []}
            continue
        if cur is not None:
            if ln.startswith(".Lfunc_end"):
                cur = None
                continue
            kernels[cur]["body"].append(ln)
    # metadata
    meta = {}
    for ln in lines:
        m = re.match(r"\s+\.(vgpr_count|agpr_count|sgpr_count|private_segment_fixed_size|name):\s+(\S+)", ln)
        if m:
            key, val = m.group(1), m.group(2)
            if key == "name":
                cur = val
                meta.setdefault(cur, {})
            elif cur is not None:
                meta.setdefault(cur, {})[key] = val
    names = list(kernels)
    dem = dict(zip(names, demangle(names)))
    for k in names:
        d = dem[k]
        if subs and not all(s in d or s in k for s in subs):
            continue
        cnt = collections.Counter()
        ops = collections.Counter()
        for ln in kernels[k]["body"]:
            t = ln.strip()
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            op = t.split()[0]
            c = classify(op)
            cnt[c] += 1
            ops[op] += 1
        md = meta.get(k, {})
        vg = int(md.get("vgpr_count", 0))
        ag = int(md.get("agpr_count", 0))
        tot = vg + ag
        occ = 8 if tot <= 64 else 512 // (((tot + 7) // 8) * 8) if tot else 8
        valu = sum(cnt[c] for c in ("valu_f64", "valu_other", "valu_mov", "dpp", "lane_xfer"))
        print(f"{d}")
        print(f"  vgpr {vg} agpr {ag} sgpr {md.get('sgpr_count')} scratch {md.get('private_segment_fixed_size')} "
              f"B  -> {min(occ, 8)} waves/SIMD")
        print(f"  VALU total {valu}: " + ", ".join(f"{c} {cnt[c]}" for c in
                                                 ("valu_f64", "valu_other", "valu_mov", "dpp", "lane_xfer")))
        print("  other: " + ", ".join(f"{c} {n}" for c, n in sorted(cnt.items()) if not c.startswith(("valu", "dpp",
                                                                                                      "lane"))))
        if "-v" in sys.argv:
            pass
        top = ", ".join(f"{o} {n}" for o, n in ops.most_common(30))
        print(f"  top: {top}")


if __name__ == "__main__":
    main()
