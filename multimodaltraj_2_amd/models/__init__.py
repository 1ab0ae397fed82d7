"""Model classes with the reference's signatures (models/*.py)."""
