"""platform"""
