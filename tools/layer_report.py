"""Per-layer timing report from a rocprofv3 kernel trace of bench.py (dev tool).

    python tools/layer_report.py <kernel_trace.csv> <frames_per_step> [--layers]

Maps the kernels of one forward (the second to last) onto the BODY_25 conv/pool layers; a
conv1_fused_kernel launch stands for conv1_1 + conv1_2 + pool1_stage1, a conv_head_kernel launch for a
stage's Mconv6 + Mconv7.
"""
import csv
import re
import sys

sys.path.insert(0, '.')
from oracle import body25  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
per_layer = '--layers' in sys.argv
ks = [r for r in rows if ('conv' in r['Kernel_Name'] and 'kernel' in r['Kernel_Name'])
      or 'maxpool' in r['Kernel_Name']]
starts = [i for i, r in enumerate(ks) if 'conv1_fused' in r['Kernel_Name'] or 'conv_image' in r['Kernel_Name']]
fw = ks[starts[-2]:starts[-1]]
L = [l for l in body25.layers() if l['type'] in ('Convolution', 'Pooling')]
H = [368, 184, 92, 46]
W = [656, 328, 164, 82]


def flops(l, lvl):
    return 2 * frames * H[lvl] * W[lvl] * l['num_output'] * l['cin'] * l['kernel_size'] ** 2


lvl = 0
tot = 0
byn = {}
li = 0
for r in fw:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    name = r['Kernel_Name']
    if 'conv1_fused' in name:   # conv1_1 + conv1_2 + pool1
        fl = flops(L[0], 0) + flops(L[1], 0)
        key = ('conv1_1+conv1_2+pool1', 3, 0)
        li += 3
        lvl = 1
        if per_layer:
            print('%-28s %8.1f us %7.1f TF/s' % (key[0], d, fl / d / 1e6))
    elif 'conv_head' in name:   # Mconv6 (1x1, PReLU) + Mconv7 (1x1) of one stage
        l6, l7 = L[li], L[li + 1]
        li += 2
        fl = flops(l6, lvl) + flops(l7, lvl)
        key = ('Mconv6+Mconv7 N1=%d' % l6['num_output'], 1, lvl)
        if per_layer:
            print('%-28s cin=%4d mid=%4d cout=%4d k=1 lvl=%d %8.1f us %7.1f TF/s' %
                  (l6['name'] + '+7', l6['cin'], l6['num_output'], l7['num_output'], lvl, d, fl / d / 1e6))
    else:
        l = L[li]
        li += 1
        if l['type'] == 'Pooling':
            lvl += 1
            if per_layer:
                print('%-28s %8.1f us' % (l['name'], d))
            tot += d
            continue
        fl = flops(l, lvl)
        key = (l['num_output'], l['kernel_size'], lvl)
        m8 = re.search(r'conv3w8_kernel<\d+, \d+, (true|false)', name)
        pooled = bool(m8) and m8.group(1) == 'true'   # conv3w8 POOL: the next pool ran inside
        if pooled:
            key = ('N=%4d k=%d lvl=%d +pool' % key, 3, lvl)
        if per_layer:
            print('%-28s cin=%4d cout=%4d k=%d lvl=%d %8.1f us %7.1f TF/s%s' %
                  (l['name'], l['cin'], l['num_output'], l['kernel_size'], lvl, d, fl / d / 1e6,
                   ' (+ %s)' % L[li]['name'] if pooled else ''))
        if pooled:
            li += 1
            lvl += 1
    tot += d
    a = byn.setdefault(key, [0, 0, 0])
    a[0] += d
    a[1] += fl
    a[2] += 1
for k, (d, fl, n) in sorted(byn.items(), key=lambda kv: -kv[1][0]):
    label = k[0] if isinstance(k[0], str) else 'N=%4d k=%d lvl=%d' % k
    print('%-24s n=%3d  %9.1f us  %7.1f TF/s' % (label, n, d, fl / d / 1e6))
print('total CNN us (convs + pools)', round(tot, 1))
