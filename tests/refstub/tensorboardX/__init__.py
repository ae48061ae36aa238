class SummaryWriter:
    def __init__(self,*a,**k): pass
    def __getattr__(self,k): return lambda *a, **kw: None
