"""Server plugins — drop-ins for the reference's servers/*.py."""
