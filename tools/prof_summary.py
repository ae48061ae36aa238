"""Group a rocprofv3 kernel_stats.csv into kernel families (per learner iteration)."""
import csv
import re
import sys
from collections import defaultdict

rules = [
    (r'^Cijk_', 'hipBLASLt GEMM'),
    (r'naive_conv', 'MIOpen naive conv (find / fallback)'),
    (r'grouped_conv_fwd', 'MIOpen CK conv fwd'), (r'grouped_conv_bwd_data', 'MIOpen CK conv bwd-data'),
    (r'bwd_weight', 'MIOpen CK conv wrw'),
    (r'igemm_fwd', 'MIOpen conv fwd'), (r'igemm_bwd', 'MIOpen conv bwd-data'), (r'igemm_wrw', 'MIOpen conv wrw'),
    (r'batched_transpose', 'MIOpen NCHW<->NHWC transpose'),
    (r'as::', 'applestar native'),
    (r'copy_kernel|direct_copy|CatArray|copyBuffer', 'copies / casts / cat'),
    (r'reduce_kernel|sum_functor', 'torch reductions'),
    (r'softmax', 'torch softmax'),
    (r'max_pool', 'torch maxpool'),
    (r'upsample', 'torch upsample'),
    (r'elementwise|Functor|SubTensor|fill|Fill|clamp|where|masked', 'torch elementwise'),
    (r'index|scatter|gather|sum_and_scatter', 'torch index/scatter'),
    (r'multi_tensor_apply|Fused', 'optimizer'),
]


def family(name: str) -> str:
    for pat, f in rules:
        if re.search(pat, name):
            return f
    return 'other'


def main():
    path = sys.argv[1]
    iters = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    rows = list(csv.DictReader(open(path)))
    fam = defaultdict(lambda: [0.0, 0])
    for r in rows:
        key = family(r['Name'])
        fam[key][0] += float(r['TotalDurationNs']) / 1e6 / iters
        fam[key][1] += int(r['Calls']) / iters
    tot = sum(v[0] for v in fam.values())
    print(f'total kernel time per iteration: {tot:.1f} ms')
    for k, (ms, calls) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f'  {ms:7.2f} ms  {100*ms/tot:5.1f}%  {calls:7.0f} launches  {k}')


if __name__ == '__main__':
    main()
