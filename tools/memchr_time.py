"""Host cost of the NUL scan a host-pointer build does (libc memchr over the string), on the
machine it runs on (diagnostic)."""
import ctypes
import os
import sys
import time

libc = ctypes.CDLL(None)
libc.memchr.restype = ctypes.c_void_p
libc.memchr.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_size_t]
for mb in (10, 100):
    b = os.urandom(mb << 20).replace(b"\0", b"A")
    for _ in range(3):
        libc.memchr(b, 0, len(b))
    t = time.perf_counter()
    for _ in range(20):
        libc.memchr(b, 0, len(b))
    print(f"memchr {mb} MB: {(time.perf_counter() - t) / 20 * 1e3:.3f} ms", flush=True)
sys.exit(0)
