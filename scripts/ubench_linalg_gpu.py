"""Timing of the PT generator's decompositions (ptgen._compress: QR of (c, P c') tails, SVD of (c P, c')) on the GPU
through torch.linalg (rocSOLVER) vs numpy on the host, at the biexciton default sizes (c up to 3 x 155, P = 5)."""
import time

import numpy as np
import torch


def bench(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


rng = np.random.default_rng(0)
for (m, n) in [(465, 775), (775, 465), (320, 320), (192, 960), (960, 192)]:
    A = rng.normal(size=(m, n)) + 1j * rng.normal(size=(m, n))
    At = torch.from_numpy(A).cuda()
    t_qr_g = bench(lambda: torch.linalg.qr(At.mH), 10)
    t_svd_g = bench(lambda: torch.linalg.svd(At, full_matrices=False), 5)
    t_qr_c = bench(lambda: np.linalg.qr(A.conj().T), 5)
    t_svd_c = bench(lambda: np.linalg.svd(A, full_matrices=False), 5)
    print(f"{m}x{n}: qr gpu {t_qr_g:.2f} ms cpu {t_qr_c:.2f} ms | svd gpu {t_svd_g:.2f} ms cpu {t_svd_c:.2f} ms", flush=True)
# batched: the nl = 3 blocks of a stacked site are independent before the merge
B = torch.from_numpy(rng.normal(size=(16, 155, 775)) + 1j * rng.normal(size=(16, 155, 775))).cuda()
print("batched 16 x 155x775 svd gpu %.2f ms" % bench(lambda: torch.linalg.svd(B, full_matrices=False), 3))
