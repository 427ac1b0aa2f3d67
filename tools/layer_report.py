"""Per-layer timing report from a rocprofv3 kernel trace of bench.py (dev tool)."""
import csv, sys
sys.path.insert(0, '.')
from oracle import body25
rows = list(csv.DictReader(open(sys.argv[1])))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
ks = [r for r in rows if 'conv' in r['Kernel_Name'] and 'kernel' in r['Kernel_Name'] or 'maxpool' in r['Kernel_Name']]
L = [l for l in body25.layers() if l['type'] in ('Convolution', 'Pooling')]
per = len(L)
nfw = len(ks) // per
fw = ks[per * (nfw - 2): per * (nfw - 1)]
lvl = 0; H = [368, 184, 92, 46]; W = [656, 328, 164, 82]
tot = 0; byn = {}
for l, r in zip(L, fw):
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    if l['type'] == 'Pooling':
        lvl += 1; continue
    fl = 2 * frames * H[lvl] * W[lvl] * l['num_output'] * l['cin'] * l['kernel_size'] ** 2
    tot += d
    k = (l['num_output'], l['kernel_size'], lvl)
    a = byn.setdefault(k, [0, 0, 0]); a[0] += d; a[1] += fl; a[2] += 1
for k, (d, fl, n) in sorted(byn.items(), key=lambda kv: -kv[1][0]):
    print('N=%4d k=%d lvl=%d  n=%3d  %8.1f us  %6.1f TF/s' % (k[0], k[1], k[2], n, d, fl / d / 1e6))
print('total conv us', round(tot, 1))
