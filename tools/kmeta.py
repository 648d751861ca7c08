"""Register / spill / LDS summary of every kernel in a hipcc --save-temps gfx950 .s file.

    python tools/kmeta.py file.s [substring]"""
import re
import sys


def main(path, sub=''):
    txt = open(path).read()
    meta = txt[txt.index('amdhsa.kernels:'):]
    for blk in re.split(r'\n  - ', meta)[1:]:
        name = re.search(r'\.name:\s+(\S+)', blk)
        if not name or sub not in name.group(1):
            continue
        f = {k: re.search(r'\.' + k + r':\s+(\S+)', blk) for k in
             ('vgpr_count', 'agpr_count', 'vgpr_spill_count', 'sgpr_count', 'sgpr_spill_count',
              'group_segment_fixed_size', 'private_segment_fixed_size')}
        print(name.group(1), ' '.join(f'{k}={v.group(1)}' for k, v in f.items() if v))


if __name__ == '__main__':
    main(*sys.argv[1:])
