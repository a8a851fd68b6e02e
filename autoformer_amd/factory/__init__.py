"""MI355X-native drop-ins for /root/reference/factory (plugin modules looked up by
``importlib.import_module(f"factory.{name}")`` in the reference trainers)."""
