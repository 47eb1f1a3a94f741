#pragma once
#include "../emu_hip.hpp"
