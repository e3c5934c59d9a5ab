"""chain"""
