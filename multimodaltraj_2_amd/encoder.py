"""encoder.py of the reference holds a single comment ("TODO encoder for head
pose and relative distance"); there is nothing to reproduce."""
