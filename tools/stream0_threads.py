"""Are two host threads' "default stream" launches one queue?  (diagnostic, GPU)

Thread A queues a ~0.5 s device sleep on torch's current (default) stream; thread B then queues a small
op on its current stream and waits for that stream: if B's wait takes ~0.5 s the default stream is one
queue for both threads (legacy null stream), if it returns at once the threads have separate queues.
Also libgsr's view of stream 0: B waits with hipStreamSynchronize(0) through ctypes.
"""
import ctypes
import threading
import time

import torch


def main():
    torch.cuda.init()
    x = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    res = {}

    def a():
        torch.cuda._sleep(1_200_000_000)

    def b(mode):
        t0 = time.time()
        if mode == "torch":
            x.add_(1)
            torch.cuda.current_stream().synchronize()
        else:
            hip.hipStreamSynchronize(ctypes.c_void_p(0))
        res[mode] = time.time() - t0

    for mode in ("torch", "hip0"):
        torch.cuda.synchronize()
        ta = threading.Thread(target=a)
        ta.start(); ta.join()
        t0 = time.time()
        tb = threading.Thread(target=b, args=(mode,))
        tb.start(); tb.join()
        torch.cuda.synchronize()
        print(f"{mode}: thread B waited {res[mode]:.3f} s (total {time.time() - t0:.3f} s); "
              f"stream handle in B: {torch.cuda.current_stream().cuda_stream:#x}", flush=True)


if __name__ == "__main__":
    main()
