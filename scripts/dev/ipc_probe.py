"""Development: does CUDA-tensor IPC (hipIpcGetMemHandle / hipIpcOpenMemHandle) work
between two processes on this box's one GPU?  torch.multiprocessing shares a device
tensor through it."""
import torch
import torch.multiprocessing as mp


def child(t, q):
    t.add_(1)
    torch.cuda.synchronize()
    q.put(float(t.sum().item()))


if __name__ == "__main__":
    mp.set_start_method("spawn")
    t = torch.zeros(1 << 20, device="cuda")
    q = mp.Queue()
    p = mp.Process(target=child, args=(t, q))
    p.start()
    print("child sum", q.get(timeout=120))
    p.join(timeout=60)
    torch.cuda.synchronize()
    print("parent sees", float(t.sum().item()), "expected", float(1 << 20))
