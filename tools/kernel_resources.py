"""VGPR / SGPR / LDS / spill figures of the kernels in a hipcc `-S` listing
(make -C parallel-krylov_amd/csrc asm EPI=<n>), from the AMDHSA metadata.
Usage: python tools/kernel_resources.py <file.s> [name-regex]"""
import re
import sys


def main(path, pat="."):
    s = open(path).read()
    meta = s[s.find("amdhsa.kernels:"):]
    for blk in re.split(r"\n  - ", meta)[1:]:
        f = dict(re.findall(r"^\s*\.(\w+):\s+(\S+)", blk, re.M))
        name = f.get("name", "?")
        if not re.search(pat, name):
            continue
        vg = int(f.get("vgpr_count", 0))
        waves = min(8, 512 // max(8, (vg + 7) // 8 * 8))
        print(f"{name[:90]:90s} vgpr {vg:3d} ({waves} waves/SIMD) sgpr {f.get('sgpr_count')} "
              f"lds {f.get('group_segment_fixed_size')} spill {f.get('vgpr_spill_count')}")


if __name__ == "__main__":
    main(*sys.argv[1:])
