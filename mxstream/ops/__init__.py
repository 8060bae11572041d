"""mxstream.ops."""
