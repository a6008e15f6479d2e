"""Instruction mix of a kernel between the MOX_ISA_MARKS comment markers.

Usage: python tools/isa_regions.py <file.s> [kernel-substring]
Prints, per region (text between '; <MARK>' comments, in order of appearance),
the static count of VALU (v_), SALU (s_), LDS (ds_) and global instructions.
Static counts: loops are counted once (read the region's loop structure next to
it).  Build the .s with:
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=max-memory-clause \
        -DMOX_ISA_MARKS --cuda-device-only -S map-oxidize_amd/csrc/mox_kernels.hip -o /tmp/k.s
"""
import re
import sys


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "k_map"
    lines = open(path).read().splitlines()
    inside = False
    region = "entry"
    counts = {}
    order = []
    for ln in lines:
        if re.match(r"^_Z\w*:", ln) or re.match(r"^\w+:\s*;\s*@", ln):
            inside = want in ln.split(":")[0]
            region = "entry"
            continue
        if not inside:
            continue
        if ln.strip().startswith("s_endpgm"):
            inside = False
            continue
        s = ln.strip()
        m = re.match(r";\s*(DO_ROW|MARK|PASS_A)\s*(.*)", s)
        if m:
            region = (m.group(1) + " " + m.group(2)).strip()
            continue
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        cls = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_")) else "other"
        if region not in counts:
            counts[region] = {}
            order.append(region)
        counts[region][cls] = counts[region].get(cls, 0) + 1
    for r in order:
        c = counts[r]
        print(f"{r:40s} " + " ".join(f"{k}={c.get(k, 0)}" for k in ("valu", "salu", "lds", "vmem", "other")))


if __name__ == "__main__":
    main()
