"""Oracle (test infrastructure): the CenterNet node's preprocessing (centernet_node.py:90-92),
`T.Normalize(ImageNet)(T.Resize((in_h, in_w))(T.ToTensor()(frame).unsqueeze(0)))`.

torchvision is absent from this container, so T.Resize is restated from
torchvision 0.15.2 (requirements.txt:3): for a float tensor, transforms.Resize ->
functional.resize -> functional_tensor.resize, which (size differing from the image's) calls
torch.nn.functional.interpolate(img, size, mode="bilinear", align_corners=False,
antialias=False) (0.15's tensor default: antialias None -> False, with a deprecation warning);
an image already at the target size is returned unchanged. The interpolation itself is torch's
own CPU upsample_bilinear2d, run here — so this restatement is pinned to torch's kernel, and
its torchvision dispatch is PARITY UNPINNED (no torchvision to import, no reference fixture).
ToTensor = u8 / 255 in fp32 (CHW); Normalize = (x - mean) / std.
"""
import torch
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def preprocess(frames_u8: torch.Tensor, in_h: int, in_w: int) -> torch.Tensor:
    """u8 RGB frames [B, H, W, 3] -> normalised fp32 [B, 3, in_h, in_w]."""
    img = frames_u8.permute(0, 3, 1, 2).contiguous().to(torch.float32).div(255)
    if tuple(img.shape[2:]) != (in_h, in_w):
        img = F.interpolate(img, (in_h, in_w), mode="bilinear", align_corners=False, antialias=False)
    m = torch.tensor(MEAN, dtype=torch.float32).view(1, 3, 1, 1)
    s = torch.tensor(STD, dtype=torch.float32).view(1, 3, 1, 1)
    return img.sub(m).div(s)
