"""Floor of a launch inside a graph on this box: an empty-ish kernel and device copies of
the sizes the full-resolution upsampler layers move, timed like scripts/conv_sweep.py."""
import torch


def timed(fn, reps=20, iters=5):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * iters)


def main():
    dev = torch.device("cuda")
    one = torch.zeros(1, device=dev)
    print(f"tiny add (1 elt)          {timed(lambda: one.add_(1)):7.2f} us")
    for mb in (0.5, 2, 7.7, 15.4, 30.7, 61.4):
        n = int(mb * 1e6 / 4)
        x = torch.randn(n, device=dev)
        y = torch.empty_like(x)
        t = timed(lambda: y.copy_(x))
        print(f"copy {mb:5.1f} MB -> {mb:5.1f} MB  {t:7.2f} us  ({2 * mb * 1e6 / (t * 1e-6) / 1e9:7.1f} GB/s)")


if __name__ == "__main__":
    main()
