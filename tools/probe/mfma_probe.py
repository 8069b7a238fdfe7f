import ctypes, os, sys, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_probe.so"))
dev = torch.device("cuda:0")
ok = True
for which, (m, n, k) in ((16, (16, 16, 32)), (32, (32, 32, 16))):
    A = torch.randint(-4, 5, (m, k), device=dev).to(torch.bfloat16)
    B = torch.randint(-4, 5, (k, n), device=dev).to(torch.bfloat16)   # asymmetric
    D = torch.zeros(m, n, device=dev)
    rc = lib.launch_probe(which, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(D.data_ptr()),
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    ref = A.float() @ B.float()
    good = torch.equal(D, ref)
    ok &= good
    print(f"mfma {which}: rc={rc} exact={good} maxdiff={(D-ref).abs().max().item()}")
sys.exit(0 if ok else 1)
