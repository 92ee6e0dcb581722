"""Diagnostic: hipMemsetAsync captured into a hipGraph (torch.cuda.graph), replayed over a buffer
refilled with 0xFF between replays: which bytes the memset node leaves non-zero, by size."""
import ctypes

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    hip.hipMemsetAsync.restype = ctypes.c_int
    for nbytes in (2048, 2064, 2080, 4112, 8192, 16, 48):
        buf = torch.full((nbytes + 256,), 0xFF, dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                st = hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, nbytes, ctypes.c_void_p(s.cuda_stream))
        torch.cuda.current_stream().wait_stream(s)
        for rnd in range(3):
            buf.fill_(0xFF)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            h = buf.cpu()
            bad = (h[:nbytes] != 0).nonzero().flatten().tolist()
            over = (h[nbytes:] != 0xFF).nonzero().flatten().tolist()
            print(f"size {nbytes} rnd {rnd} status {st}: nonzero inside {len(bad)} "
                  f"(first {bad[:4]}, last {bad[-4:]}), touched beyond {len(over)}", flush=True)
        # eager for comparison
        buf.fill_(0xFF)
        hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, nbytes, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        h = buf.cpu()
        print(f"size {nbytes} eager: nonzero inside {int((h[:nbytes] != 0).sum())}", flush=True)
        del g


if __name__ == "__main__":
    main()
