"""DynamicFusion loop over this package's GPU components (reference apps/fusion/)."""
from .pipeline import (FusionParameters, FusionPipeline, FrameResult, GraphGenerationMode,  # noqa: F401
                       MeshExtractionWeightThresholdingMode, TrackingMethod, TrackingSpanMode)
