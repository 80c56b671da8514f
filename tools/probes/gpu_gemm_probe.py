import torch, time
dev = "cuda"
def bench(M, K, N, reps=50):
    a = torch.randn(M, K, device=dev); b = torch.randn(K, N, device=dev)
    for _ in range(5): c = a @ b
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(reps): c = a @ b
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / reps
    return 2 * M * K * N / dt / 1e12
for lib in ("cublas", "cublaslt"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print(lib, "unavailable", e); continue
    print(lib, torch.backends.cuda.preferred_blas_library(), {f"{M}x{K}x{N}": round(bench(M, K, N), 1) for (M, K, N) in
          [(32768, 352, 256), (32768, 256, 256), (32768, 352, 512), (256, 32768, 352), (256, 32768, 256), (32768, 256, 352), (4096, 352, 512)]})
