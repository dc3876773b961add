from .unet import UNet3D, ConvBlock3D, DownBlock3D, UpBlock3D, build_unet3d  # noqa: F401
from .dual_encoder import DualEncoder, CrossModalAttention, build_dual_encoder  # noqa: F401
from .swin_unetr import SwinUNETR, build_swin_unetr  # noqa: F401
