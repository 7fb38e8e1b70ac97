"""v1/threads (reference): only ``pipeline`` is provided."""
