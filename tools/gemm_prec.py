import torch
print("allow_tf32", torch.backends.cuda.matmul.allow_tf32, torch.get_float32_matmul_precision())
g = torch.Generator().manual_seed(0)
a = torch.randn(100000, 64, generator=g); b = torch.randn(100000, 32, generator=g)
want = (a.double().t() @ b.double())
for prec in ("highest", "high"):
    torch.set_float32_matmul_precision(prec)
    got = (a.cuda().t() @ b.cuda()).cpu().double()
    print(prec, float((got - want).norm() / want.norm()))
    x = torch.randn(4096, 64, generator=g); w = torch.randn(32, 64, generator=g)
    y = torch.nn.functional.linear(x.cuda(), w.cuda()).cpu().double()
    print(prec, "linear", float((y - x.double() @ w.double().t()).norm() / y.norm()))
