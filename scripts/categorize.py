"""Group a prof_diff.py kernel summary into categories (ms/step)."""
import re
import sys

CATS = [('ours conv fwd', r'conv_fwd_kernel<[^>]*, [0-57], (true|false)>|conv_fwd_(glds|halo)_kernel<\d+, \d+, \d+, [0-57], \d+>|fh2_fwd'),
        ('ours dgrad', r'conv_fwd_kernel<[^>]*, [68], |conv_fwd_(glds|halo)_kernel<\d+, \d+, \d+, [68], \d+>|fh2_dgrad'),
        ('ours split', r'split_hilo'),
        ('ours conv fwd', r'conv_enc64|stem_conv_fwd'),
        # the 7x7 stem's weight gradient: per-workgroup partials + their fixed-order reduce
        ('ours wgrad', r'stem_conv_wgrad|stem_wgrad_reduce'),
        ('ours wgrad', r'fh2_wgrad'),
        ('ours wgrad', r'conv_wgrad'),
        ('encoder norm', r'norm_(bwd_)?(stats|apply|finalize|reduce_finalize)|partial_reduce|add_relu|relu_mask'),
        # hipBLASLt: the two GEMMs of the all-pairs correlation backward (dF1 = dC F2, dF2 = dC^T F1)
        ('corr gemm', r'Cijk_'),
        ('update ew', r'f1_patch|sum_bf16'),
        ('miopen conv', r'igemm|grouped_conv|naive_conv|gemm|Conv'), ('transpose', r'transpose'),
        ('bn/norm', r'batch_norm|BatchNorm|InstanceNorm|instance_norm|welford|Norm'),
        ('corr', r'corr_'), ('reduce', r'reduce_kernel'),
        ('elementwise', r'elementwise|vectorized|SubTensor|OpTensor|Cast|copy_kernel|unrolled'),
        ('corr', r'corr_'), ('upsample', r'convex'), ('update ew', r'relu_bwd|gru_|flow_prep'),
        ('copy', r'copyBuffer'), ('loss', r'seq_loss'), ('adam', r'adam|Adam|multi_tensor')]
tot = {}
phase_tot = {}
for line in open(sys.argv[1]):
    if not re.match(r'\s*[\d.]+%', line):
        continue
    parts = line.split(None, 4)
    ms, name = float(parts[3]), parts[4]
    # prof_diff.py --phases prefixes '[decode] ' / '[encoder] ': our conv kernels serve both the
    # update block (decode) and the encoders, so their categories are split by phase
    m = re.match(r'\[(decode|encoder)\] (.*)', name)
    phase = None
    if m:
        phase, name = m.group(1), m.group(2)
        phase_tot[phase] = phase_tot.get(phase, 0) + ms
    # fp16 (EPI_F16 = 16) and split-fp32 (EPI_SPL = 32) instantiations: the base epilogue's category
    name = re.sub(r'(conv_fwd_(?:glds|halo)_kernel<\d+, \d+, \d+, )(\d+)',
                  lambda k: k.group(1) + str(int(k.group(2)) & 15), name)
    for c, pat in CATS:
        if re.search(pat, name):
            if phase and c.startswith('ours'):
                c = c.replace('ours', 'update-block' if phase == 'decode' else 'encoder')
            tot[c] = tot.get(c, 0) + ms
            break
    else:
        tot['other'] = tot.get('other', 0) + ms
for c, v in sorted(tot.items(), key=lambda x: -x[1]):
    print('%-15s %7.2f' % (c, v))
print('%-15s %7.2f' % ('total', sum(tot.values())))
for p, v in sorted(phase_tot.items()):
    print('%-15s %7.2f' % ('phase ' + p, v))
