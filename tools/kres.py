"""Per-kernel resource usage of one HIP translation unit (gfx950):
VGPRs, SGPRs, spills, LDS, occupancy -- from clang's kernel-resource-usage
remarks.  Used to check that a refactor leaves the batch kernels' code
unchanged in what matters (registers, spills, occupancy).

    python tools/kres.py orb_slam_fusion_amd/csrc/orb_kernels.hip [-D...]
"""
import re
import subprocess
import sys


def resources(src, extra=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
           "--offload-device-only", "-c", "-Rpass-analysis=kernel-resource-usage", src, "-o", "/dev/null", *extra]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = rows.setdefault(val, {})
        elif cur is not None:
            cur[key] = val
    return rows


def main():
    rows = resources(sys.argv[1], sys.argv[2:])
    cols = ["VGPRs", "AGPRs", "TotalSGPRs", "SGPRs Spill", "VGPRs Spill", "LDS Size [bytes/block]",
            "Occupancy [waves/SIMD]"]
    print("kernel".ljust(60), *[c.split(" [")[0][:10].rjust(10) for c in cols])
    for name, r in sorted(rows.items()):
        short = re.sub(r"^_ZN6orbgpu\d+", "", name)[:58]
        print(short.ljust(60), *[str(r.get(c, "-")).rjust(10) for c in cols])


if __name__ == "__main__":
    main()
