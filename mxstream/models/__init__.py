"""mxstream.models."""
