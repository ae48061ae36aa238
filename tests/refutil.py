"""Helpers to execute the *reference* implementation (read-only source under /root/reference) for
parity tests.  Third-party modules the reference imports but this image lacks (lz4, absl, cv2,
s2clientprotocol, tensorboardX, easydict) are replaced by tiny stubs in tests/refstub; nothing of the
reference is copied.  Tests using this skip when the reference tree is absent (e.g. on GPU boxes)."""
import os
import sys

REF = os.environ.get('APPLESTAR_REFERENCE', '/root/reference')
STUB = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'refstub')


def reference_available() -> bool:
    return os.path.isdir(os.path.join(REF, 'distar'))


def import_reference():
    import numpy as np
    for name, typ in (('int', int), ('float', float), ('bool', bool)):
        if not hasattr(np, name):
            setattr(np, name, typ)
    for p in (STUB, REF):
        if p not in sys.path:
            sys.path.append(p)
    import distar.agent.default.model.model as ref_model  # noqa
    return ref_model
