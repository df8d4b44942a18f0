from .rendering_alignment_optimizer import (PenaltyFunction, RenderingAlignmentOptimizer,  # noqa: F401
                                            RenderingAlignmentParameters)
