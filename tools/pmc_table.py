"""Per-dispatch counter table of a rocprofv3 --pmc run: kernel (short name), grid, and each counter.

    python tools/pmc_table.py <counter_collection.csv> [name-substring]
"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    sub = sys.argv[2] if len(sys.argv) > 2 else ''
    table = collections.OrderedDict()
    for r in rows:
        name = r.get('Kernel_Name', '')
        if sub not in name:
            continue
        key = (int(r.get('Dispatch_Id', 0)), re.sub(r'\(.*', '', name)[-60:], r.get('Grid_Size', ''))
        table.setdefault(key, {})[r['Counter_Name']] = float(r['Counter_Value'])
    names = sorted({c for v in table.values() for c in v})
    print('dispatch kernel grid ' + ' '.join(names))
    for (d, k, g), v in table.items():
        print(d, k, g, ' '.join(f'{v.get(c, 0):.0f}' for c in names))


if __name__ == '__main__':
    main()
