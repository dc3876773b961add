from .sliding_window import sliding_window_inference, window_starts

__all__ = ["sliding_window_inference", "window_starts"]
