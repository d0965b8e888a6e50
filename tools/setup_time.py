import sys, time, ctypes as C
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from amg_amd import _native as N
n = int(sys.argv[1])
M = N.generate(7, n)
t = time.perf_counter()
H = N.Hierarchy(M)
print("setup", time.perf_counter() - t, file=sys.stderr)
