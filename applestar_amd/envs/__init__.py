"""Environments: the real SC2 adapter (needs the SC2 binary + ``s2clientprotocol``) and FakeSC2Env."""
from __future__ import annotations


def sc2_available() -> bool:
    try:
        import s2clientprotocol  # noqa: F401
        from .sc2_env import find_sc2_binary
        return find_sc2_binary() is not None
    except Exception:  # noqa: BLE001
        return False


def make_env(cfg):
    env = cfg['env'] if 'env' in cfg else cfg
    fake = env.get('fake', None)
    if fake or (fake is None and not sc2_available()):
        from .fake_env import FakeSC2Env
        return FakeSC2Env(cfg)
    from .sc2_env import SC2Env
    return SC2Env(cfg)
