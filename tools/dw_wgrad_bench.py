"""Time sdp_dw_wgrad alone at the XL training shape (B 120, 16 x 16, C 768, k 7) on the GPU."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sdp-net_amd"))
import sdpnet_hip as sp  # noqa: E402


def main():
    B, H, W, C, k = 120, 16, 16, 768, 7
    a = torch.randn(B * H * W, C, device="cuda").to(torch.bfloat16)
    dy = torch.randn(B * H * W, C, device="cuda").to(torch.bfloat16)
    nch = sp.lib().sdp_dw_wgrad_chunks(B)
    part = torch.empty(nch, C * k * k, dtype=torch.float32, device="cuda")
    args = (1, a.data_ptr(), C, 0, 0, 0, dy.data_ptr(), C, 0, 0, 0, B, H, W, C, k, part.data_ptr(), None)
    for _ in range(3):
        sp.lib().sdp_dw_wgrad(*args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 50
    for _ in range(n):
        sp.lib().sdp_dw_wgrad(*args)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    mb = 2 * a.numel() * 2 / 1e6
    print(f"dw_wgrad B{B} {H}x{W} C{C} k{k}: {us:.1f} us, {mb:.0f} MB -> {mb / us:.2f} TB/s")


if __name__ == "__main__":
    main()
