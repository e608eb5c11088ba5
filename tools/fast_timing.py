"""Summarise the performance kernel's per-wave cycle stamps (a library built
with DP_EXTRA_FLAGS=-DDP_FAST_TIMING prints one "TM blk ..." line per sampled
wave): share of the wave's cycles per phase, summed over every printed line.

    python tools/fast_timing.py gpurun_out/timing.log
"""
import re
import sys

# TMARK indices in dp_fast.hip
NAMES = {
    0: "dequeue / child pose", 1: "frame", 2: "staging geometry", 3: "tile DMA issue", 4: "DMA wait",
    5: "CG bookkeeping", 6: "InitRelatedImages", 7: "filter frame", 8: "filter masks / finish",
    9: "write-back", 10: "eval record build", 11: "sampling passes", 12: "NCC finish", 14: "objective sum",
    15: "CG step",
}


def main(path):
    tot = [0] * 16
    total = patches = lines = 0
    for ln in open(path, errors="replace"):
        if not ln.startswith("TM blk"):
            continue
        f = dict(re.findall(r"(\w+) (\d+)", ln))
        lines += 1
        patches += int(f["patches"])
        total += int(f["total"])
        for k in range(16):
            tot[k] += int(f[f"r{k}"])
    if not lines:
        sys.exit("no TM lines")
    print(f"{lines} waves, {patches} patches, {total / max(patches, 1):.0f} cycles per patch")
    for k in sorted(range(16), key=lambda k: -tot[k]):
        if tot[k]:
            print(f"  r{k:<2} {NAMES.get(k, '?'):24s} {100.0 * tot[k] / total:5.1f}%  {tot[k] / patches:8.0f} cyc/patch")


if __name__ == "__main__":
    main(sys.argv[1])
