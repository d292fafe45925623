"""native"""
