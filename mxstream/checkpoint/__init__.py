"""mxstream.checkpoint."""
