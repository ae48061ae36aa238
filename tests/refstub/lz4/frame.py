def compress(x): return x
def decompress(x): return x
