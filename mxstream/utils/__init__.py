"""mxstream.utils."""
