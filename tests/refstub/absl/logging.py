def info(*a, **k): pass
def warning(*a, **k): pass
def error(*a, **k): pass
