// tests/walnut_stub/Walnut/EntryPoint.h -- TEST STUB: the driver (driver.cpp) is the entry point.
#pragma once
#include "Walnut/Application.h"
