"""Instruction mix of a kernel's innermost loop(s) in a hipcc -S listing:
from each 'Loop Header' label to the branch back to it.
Usage: python tools/loop_mix.py <file.s> <kernel-symbol-regex>"""
import collections
import re
import sys


def main(path, pat):
    L = open(path).read().splitlines()
    for st, l in enumerate(L):
        if not (re.match(r"^[\w.]+:", l) and re.search(pat, l.split(":")[0])):
            continue
        end = next(i for i in range(st, len(L)) if L[i].startswith(".Lfunc_end"))
        body = L[st:end]
        for h, l2 in enumerate(body):
            if "Loop Header" not in l2:
                continue
            lab = l2.split(":")[0]
            e = max(i for i, x in enumerate(body) if re.search(r"s_(c)?branch\w* " + re.escape(lab) + "$", x.strip()))
            c = collections.Counter()
            for x in body[h:e + 1]:
                x = x.strip()
                if x and not x.startswith((".", ";")) and not x.endswith(":"):
                    c[x.split()[0]] += 1
            v = sum(n for k, n in c.items() if k.startswith("v_"))
            print(f"{l.split(':')[0][:100]}\n  loop {lab}: {e - h} lines, VALU {v}, "
                  f"LDS {sum(n for k, n in c.items() if k.startswith('ds_'))}, "
                  f"VMEM {sum(n for k, n in c.items() if k.startswith(('global_', 'buffer_')))}, "
                  f"SALU {sum(n for k, n in c.items() if k.startswith('s_'))}")
            print("  " + " ".join(f"{k}:{n}" for k, n in c.most_common(24)))


if __name__ == "__main__":
    main(*sys.argv[1:])
