"""VGPR / SGPR / scratch / LDS use of every kernel in a hipcc -S output (gfx950): spills into scratch
(private segment) in a hot kernel are a regression to catch before a GPU run.

usage: python tools/isa_resources.py ke.s [name-filter]
"""
import re
import sys


def main():
    src = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", src, re.S):
        name, body = m.group(1), m.group(2)
        get = lambda k: int(re.search(r"\.amdhsa_" + k + r" (\d+)", body).group(1))  # noqa: E731
        short = re.sub(r"^_ZN2ke\d+", "", name)[:60]
        if filt in name:
            print(f"{short:60s} vgpr={get('next_free_vgpr'):4d} sgpr={get('next_free_sgpr'):4d} "
                  f"scratch={get('private_segment_fixed_size'):5d} lds={get('group_segment_fixed_size'):6d}")


if __name__ == "__main__":
    main()
