"""Seeded synthetic event windows in the reference's collate layout
(``dataloader/base.py:261-278``; SURVEY 8(d) "Synthetic input"):
  event_list [B,N,4] (ts, y, x, p) with ts sorted and normalised to [0,1]
  (``dataloader/base.py:94-96``), p in {-1,+1}; event_list_pol_mask [B,N,2];
  event_cnt [B,2,H,W] per-polarity counts (``dataloader/encodings.py:70-85``);
  event_mask [B,1,H,W] = pixel has an event.
Generated on the target device with torch ops (input plumbing, outside the hot path)."""
import torch


def make_window(B, N, H, W, generator, device):
    ys = torch.randint(0, H, (B, N), generator=generator, device=device)
    xs = torch.randint(0, W, (B, N), generator=generator, device=device)
    ts = torch.sort(torch.rand(B, N, generator=generator, device=device), dim=1).values
    lo, hi = ts[:, :1], ts[:, -1:]
    ts = (ts - lo) / (hi - lo).clamp_min(1e-12)
    pos = torch.rand(B, N, generator=generator, device=device) < 0.5
    ps = pos.float() * 2 - 1
    ev = torch.stack([ts, ys.float(), xs.float(), ps], dim=2).contiguous()
    pol = torch.stack([pos.float(), (~pos).float()], dim=2).contiguous()
    flat = (ys * W + xs) + (torch.arange(B, device=device) * (H * W)).unsqueeze(1)
    cnt = torch.zeros(B * 2 * H * W, device=device)
    ch = (~pos).long() * (H * W) + flat + (torch.arange(B, device=device) * (H * W)).unsqueeze(1)
    cnt.index_add_(0, ch.reshape(-1), torch.ones(B * N, device=device))
    cnt = cnt.view(B, 2, H, W)
    mask = (cnt.sum(1, keepdim=True) > 0).float()
    return {"event_list": ev, "event_list_pol_mask": pol, "event_cnt": cnt, "event_mask": mask,
            "event_voxel": cnt}
