"""Does a captured hipGraph run independent branches (two streams forked from the capture stream) concurrently?
Times 2 x K small, independent GEMMs (few blocks each) serial on one stream vs forked over two streams, eagerly and
captured.  Prints ms per replay; concurrency shows as the forked time approaching half the serial time."""
import torch


def main():
    dev = torch.device("cuda", 0)
    n, K = 512, 32
    a = [torch.randn(n, n, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    out = [torch.empty(n, n, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    s1 = torch.cuda.Stream(dev)

    def serial():
        for _ in range(K):
            torch.matmul(a[0], a[0], out=out[0])
            torch.matmul(a[1], a[1], out=out[1])

    def forked():
        main = torch.cuda.current_stream(dev)
        s1.wait_stream(main)
        for _ in range(K):
            torch.matmul(a[0], a[0], out=out[0])
        with torch.cuda.stream(s1):
            for _ in range(K):
                torch.matmul(a[1], a[1], out=out[1])
        main.wait_stream(s1)

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    res = {"eager_serial": timeit(serial), "eager_forked": timeit(forked)}
    for name, fn in (("graph_serial", serial), ("graph_forked", forked)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        res[name] = timeit(g.replay)
    print({k: round(v, 4) for k, v in res.items()})


if __name__ == "__main__":
    main()
