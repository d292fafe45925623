"""The three Tasks Tracker microservices and their shared host."""
