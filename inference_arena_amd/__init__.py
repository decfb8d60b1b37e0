"""inference_arena_amd — MI355X-native serving arena (YOLOv5nu -> MobileNetV2)."""
__version__ = "0.1.0"
