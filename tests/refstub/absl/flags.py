class _F:
    def __getattr__(self, k): return None
    def __call__(self, *a, **k): return self
FLAGS=_F()
def DEFINE_string(*a, **k): pass
def DEFINE_integer(*a, **k): pass
def DEFINE_bool(*a, **k): pass
def DEFINE_boolean(*a, **k): pass
def DEFINE_enum(*a, **k): pass
def DEFINE_float(*a, **k): pass
