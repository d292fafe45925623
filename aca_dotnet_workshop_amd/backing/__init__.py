"""backing"""
