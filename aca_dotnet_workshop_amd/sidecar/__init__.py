"""sidecar"""
