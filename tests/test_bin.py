"""Entry points without SC2: play on the fake env, rl/sl launch configs, Z library assembly,
resumable download against a local HTTP server."""
import http.server
import os
import threading

import pytest
import torch


def test_play_agent_vs_bot_fake_env(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    from applestar_amd.bin import play
    cfg_path = tmp_path / 'cfg.yaml'
    cfg_path.write_text(open(os.path.join(os.path.dirname(play.__file__), 'user_config.yaml')).read()
                        .replace('game_steps_per_episode: 100000', 'game_steps_per_episode: 300'))
    res = play.main(['--config', str(cfg_path), '--game_type', 'agent_vs_bot', '--cpu', '--fake-env',
                     '--map', 'KairosJunction'])
    assert len(res) == 1 and res[0]['0']['winloss'] in (-1, 0, 1)


def test_z_library_assembly():
    from applestar_amd.bin.gen_z import add_entry, z_entry
    from applestar_amd.agent.features import Features
    from applestar_amd.envs.fake_env import FakeSC2Env
    from applestar_amd.lib.game_data import BEGINNING_ORDER_ACTIONS, CUMULATIVE_STAT_ACTIONS
    env = FakeSC2Env({'env': {'player_ids': ['a', 'b'], 'random_seed': 0}})
    obs, gi, _ = env.reset()
    f = Features(gi[0], obs[0]['raw_obs'])
    steps = [{'action_info': {'action_type': torch.tensor(a), 'target_location': torch.tensor(1000 + i)}}
             for i, a in enumerate(BEGINNING_ORDER_ACTIONS[1:13] + [CUMULATIVE_STAT_ACTIONS[5]])]
    bo, cum, loc, n, loop = z_entry(f, steps, 777)
    assert n == 13 - (1 if CUMULATIVE_STAT_ACTIONS[5] not in BEGINNING_ORDER_ACTIONS else 0) or n >= 12
    assert len(bo) == 20 and len(loc) == 20 and loop == 777 and 5 in cum
    lib = {}
    add_entry(lib, 'KairosJunction', 'zerg', f.home_born_location, [bo, cum, loc, loop])
    assert lib['KairosJunction']['zerg'][str(f.home_born_location)][0][3] == 777


def test_resumable_download(tmp_path):
    pytest.importorskip('requests')
    payload = os.urandom(300000)
    (tmp_path / 'srv').mkdir()
    (tmp_path / 'srv' / 'rl_model.pth').write_bytes(payload)

    class H(http.server.SimpleHTTPRequestHandler):
        def __init__(self, *a, **k):
            super().__init__(*a, directory=str(tmp_path / 'srv'), **k)

        def log_message(self, *a):
            pass

        def send_head(self):  # minimal Range support
            rng = self.headers.get('Range')
            if not rng:
                return super().send_head()
            start = int(rng.split('=')[1].split('-')[0])
            data = payload[start:]
            self.send_response(206)
            self.send_header('Content-Length', str(len(data)))
            self.end_headers()
            import io
            return io.BytesIO(data)
    srv = http.server.ThreadingHTTPServer(('127.0.0.1', 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    from applestar_amd.bin.download_model import download
    dest = tmp_path / 'rl_model.pth'
    (tmp_path / 'rl_model.pth.part').write_bytes(payload[:123456])  # interrupted earlier
    download(f'http://127.0.0.1:{srv.server_address[1]}/rl_model.pth', str(dest), quiet=True)
    assert dest.read_bytes() == payload
    srv.shutdown()
