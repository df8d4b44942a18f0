"""DeepDeform input formats and frame datasets (reference data/)."""
from . import io, camera, frame  # noqa: F401
from .camera import StaticCenterCrop, PinholeCameraIntrinsic  # noqa: F401
from .frame import (DataSplit, DatasetType, FramePairDataset, FrameSequenceDataset, SequenceFrameDataset,  # noqa: F401
                    StandaloneFrameDataset, StaticFrameSequenceDataset, make_frame_file_name_mask)
