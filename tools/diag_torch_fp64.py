"""Diagnostic: torch fp64 elementwise math on the GPU against numpy on the host (same inputs): the
largest relative difference of each operation a covariance plug-in typically uses."""
import numpy as np
import torch

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
x = rng.uniform(0.0, 1.0, 1_000_000)
y = rng.uniform(-1.0, 1.0, 1_000_000)
g = torch.from_numpy(x).to(dev)
h = torch.from_numpy(y).to(dev)


def rel(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else a
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


print("mul", rel(g * h, x * y))
print("pow2", rel(g ** 2, x ** 2))
print("sqrt", rel(torch.sqrt(g), np.sqrt(x)))
print("exp", rel(torch.exp(-20 * g), np.exp(-20 * x)))
print("exp_sqrt", rel(torch.exp(-torch.sqrt(50 * g)), np.exp(-np.sqrt(50 * x))))
A = np.array([[400.0, 150.0], [150.0, 100.0]])
t = rng.uniform(-0.05, 0.05, (200000, 2))
tt = torch.from_numpy(t).to(dev)
print("matmul", rel(((tt @ torch.from_numpy(A).to(dev)) * tt).sum(-1), ((t @ A) * t).sum(-1)))
print("quad_elementwise", rel(A[0, 0] * tt[:, 0] ** 2 + 2 * A[0, 1] * tt[:, 0] * tt[:, 1] + A[1, 1] * tt[:, 1] ** 2,
                              A[0, 0] * t[:, 0] ** 2 + 2 * A[0, 1] * t[:, 0] * t[:, 1] + A[1, 1] * t[:, 1] ** 2))
