"""Resumable HTTP download of released checkpoints (``distar/bin/download_model.py``): a partial
``<file>.part`` is continued with a ``Range`` request, then atomically renamed.

    python -m applestar_amd.bin.download_model --name rl_model
"""
from __future__ import annotations

import argparse
import os
import sys

DEFAULT_URL = 'https://opendilab.net/download/DI-star/'
MODELS = ['rl_model.pth', 'sl_model.pth', 'Abathur.pth', 'Zagara.pth', 'Dehaka.pth']


def download(url: str, dest: str, chunk: int = 1 << 20, timeout: float = 60.0, quiet: bool = False) -> str:
    import requests
    part = dest + '.part'
    have = os.path.getsize(part) if os.path.exists(part) else 0
    headers = {'Range': f'bytes={have}-'} if have else {}
    with requests.get(url, headers=headers, stream=True, timeout=timeout) as r:
        if r.status_code == 416:  # already complete
            os.replace(part, dest)
            return dest
        r.raise_for_status()
        if have and r.status_code != 206:  # server ignored the range: restart
            have = 0
        total = int(r.headers.get('Content-Length', 0)) + have
        with open(part, 'ab' if have else 'wb') as f:
            for buf in r.iter_content(chunk):
                f.write(buf)
                have += len(buf)
                if not quiet and total:
                    sys.stdout.write(f'\r{os.path.basename(dest)}: {100.0 * have / total:5.1f}%')
                    sys.stdout.flush()
    if not quiet:
        sys.stdout.write('\n')
    os.replace(part, dest)
    return dest


def main(argv=None):
    ap = argparse.ArgumentParser(description='download_model')
    ap.add_argument('--name', default='rl_model', help='model name (rl_model, sl_model, ...)')
    ap.add_argument('--url', default=DEFAULT_URL)
    ap.add_argument('--out_dir', default=os.path.dirname(os.path.abspath(__file__)))
    args = ap.parse_args(argv)
    name = args.name if args.name.endswith('.pth') else args.name + '.pth'
    return download(args.url.rstrip('/') + '/' + name, os.path.join(args.out_dir, name))


if __name__ == '__main__':
    main()
