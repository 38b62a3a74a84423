"""snnflow -- MI355X-native (gfx950) LIFFireNet + event-warping hot path.

Drop-in for the reference's ``models.model`` (LIFFireNet family), its spiking cells,
``loss.flow.EventWarping`` and ``utils.iwe``; all compute runs in the HIP C-ABI library
``libsnnflow.so`` (include/snnflow.h).  Importing fails loudly if the library is missing.
"""
from . import _lib  # noqa: F401  (loads libsnnflow.so or raises)
from ._lib import SnnflowError, check_device_errors
from .cells import ConvLayer, Leaky, SNNtorch_ConvLIF, SNNtorch_ConvLIFRecurrent
from .norm import MPBN, TEBN
from .convlif import ConvLIF, ConvLIFRecurrent
from . import checkpoint, encodings  # noqa: F401  (checkpoint interchange, on-device event encodings)
from .loss import EventWarping
from .metrics import AAE, AAE_Filtered, AAE_Weighted, AE_ofMeans, AEE, NAAE, NEE
from .optim import ClipAdam
from .model import LIFFireFlowNet, LIFFireFlowNet_short, LIFFireNet, LIFFireNet_short
from .unet import (SpikingMultiResUNetRecurrent, SpikingRecEVFlowNet, SpikingRecurrentConvLayer,
                   SpikingResidualBlock, SpikingUpsampleConvLayer)

__all__ = ["LIFFireNet", "LIFFireNet_short", "LIFFireFlowNet", "LIFFireFlowNet_short", "SNNtorch_ConvLIF",
           "SNNtorch_ConvLIFRecurrent", "ConvLIF", "ConvLIFRecurrent", "ConvLayer", "Leaky", "EventWarping", "AEE",
           "NEE", "AAE", "NAAE", "AE_ofMeans", "AAE_Weighted", "AAE_Filtered", "SpikingRecEVFlowNet",
           "SpikingMultiResUNetRecurrent", "SpikingRecurrentConvLayer", "SpikingResidualBlock", "SpikingUpsampleConvLayer",
           "ClipAdam", "SnnflowError", "check_device_errors"]
