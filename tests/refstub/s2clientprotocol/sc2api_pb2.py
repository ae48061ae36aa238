class _Any:
    def __init__(self, *a, **k): pass
    def __getattr__(self, k): return _Any()
    def __call__(self, *a, **k): return _Any()
    def __iter__(self): return iter([])
    def __int__(self): return 0
    def __index__(self): return 0
    def __hash__(self): return 0
    def __eq__(self, o): return False
    def __lt__(self, o): return False
    def __gt__(self, o): return False
    def ParseFromString(self, *a): pass
    def Name(self, *a): return ''
def __getattr__(name):
    return _Any()


# real enum values of sc2api.proto (the reference's featurizer / agent compare against these)
Participant, Computer, Observer = 1, 2, 3                  # PlayerType
Victory, Defeat, Tie, Undecided = 1, 2, 3, 4               # Result
Terran, Zerg, Protoss, Random = 1, 2, 3, 4                 # Race (common.proto, re-exported)
