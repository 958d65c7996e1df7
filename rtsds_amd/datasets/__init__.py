"""Dataset readers (reference datasets/): file discovery and id merging as the reference;
samples are decoded to uint8 HWC tensors on the CPU (PIL) and transformed on the device by
rtsds_amd.transforms (the reference's torchvision transforms, as HIP kernels)."""
from .cityscapes import CityScapes, class_names  # noqa: F401
from .gta5 import GTA5  # noqa: F401
